// qie_index.hpp — internal definition of the reference-compatible tensor index.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

struct qie_index_entry {
    std::string name, short_name;
    int32_t layer = -1;
    int64_t off0 = 0, off1 = 0;
    std::vector<int64_t> shape;
};

struct qie_index {
    std::vector<qie_index_entry> t;
};

namespace qie {
const qie_index_entry* index_find(const qie_index* idx, const char* short_name, int layer);
}
