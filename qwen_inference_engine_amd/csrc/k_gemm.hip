// k_gemm.hip — MFMA bf16 GEMM for the prefill projections (M = prompt rows).
//
// Replaces matrix_mul (layers/src/matrix_mul.cu:165-288) for M > 8: the
// reference computes one 16x16 WMMA tile per warp with scalar 2-byte loads into
// per-warp smem and no pipelining.  Here (gfx950):
//   C[M, N] = A[M, K] . W[N, K]^T   (both operands K-contiguous, "NT")
//   * 128x128 block tile, BK = 64, 4 waves as 2x2, 64x64 per wave =
//     4x4 v_mfma_f32_16x16x32_bf16 accumulators (fp32);
//   * 16-byte global loads staged through registers into a double-buffered,
//     XOR-swizzled LDS image (chunk ^= row & 7), fragments by ds_read_b128;
//     one barrier per K-tile, next tile's global loads in flight under the
//     current tile's MFMAs;
//   * fused epilogues: bias, residual add, SwiGLU (tile columns pair gate/up
//     rows of the same output column inside one wave).
//   * blockIdx.x runs over M tiles so the blocks sharing a weight tile are
//     adjacent in dispatch order (weights streamed ~once, activations L2/MALL).
#include "qie_common.hpp"
#include "../../include/qie/qie_ops.h"

#include <map>
#include <mutex>

namespace qie {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct GemmParams {
    const uint16_t* A;
    int64_t lda;
    const uint16_t* w0;
    const uint16_t* w1;
    const uint16_t* w2;
    const uint16_t* b0;
    const uint16_t* b1;
    const uint16_t* b2;
    int64_t n0, n01;
    int64_t M, K, N;     // N = output columns
    int64_t wrows;       // total weight rows addressable (for clamping)
    uint16_t* C;
    int64_t ldc;
};

constexpr int BM = 128, BN = 128, BK = 64;

// Weight row for tile column c of block tile starting at output column n0; eb = bytes
// per weight; for fp8 (eb = 1) also the row's scale (stored after the segment's codes).
template <int EPI>
__device__ __forceinline__ const uint16_t* w_row(const GemmParams& p, int64_t nblk, int c, bool& valid, int eb,
                                                 int64_t& row, float& scale) {
    auto at = [&](const uint16_t* w, int64_t rows, int64_t r) {
        const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
        scale = eb == 1 ? reinterpret_cast<const float*>(b + rows * p.K)[r] : 1.f;
        row = r;
        return reinterpret_cast<const uint16_t*>(b + r * p.K * eb);
    };
    if constexpr (EPI == QIE_EPI_SWIGLU) {
        // 64 output columns per tile: cols [64wc, 64wc+32) gate, [64wc+32, 64wc+64) up.
        const int64_t j = nblk * 64 + 32 * (c >> 6) + (c & 31);
        valid = j < p.N;
        const int64_t jj = valid ? j : p.N - 1;
        return ((c >> 5) & 1) ? at(p.w1, p.N, jj) : at(p.w0, p.N, jj);
    } else {
        const int64_t r = nblk * BN + c;
        valid = r < p.N;
        const int64_t rr = valid ? r : p.N - 1;
        if (rr < p.n0) return at(p.w0, p.n0, rr);
        if (rr < p.n01) return at(p.w1, p.n01 - p.n0, rr - p.n0);
        return at(p.w2, p.N - p.n01, rr - p.n01);
    }
}

// fp8 weights (WT = 1, QIE_LINEAR_FP8): e4m3 codes + power-of-two row scales after the
// [rows, K] code block; a B chunk (8 weights) is one 8-byte load, decoded and scaled to
// bf16 (exact: 3 mantissa bits x 2^k) before the LDS store, so the MFMA path is the
// bf16 one at half the weight bytes.
__device__ __forceinline__ uint4 fp8x8_to_bf16(uint2 q, float sc) {
    float f[8];
    fp8x4_to_f32(q.x, f);
    fp8x4_to_f32(q.y, f + 4);
    return make_uint4(pack2(f[0] * sc, f[1] * sc), pack2(f[2] * sc, f[3] * sc), pack2(f[4] * sc, f[5] * sc),
                      pack2(f[6] * sc, f[7] * sc));
}

template <int EPI, int WT>
__global__ __launch_bounds__(256) void gemm_kernel(GemmParams p) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint16_t* As = reinterpret_cast<uint16_t*>(smem);                 // [2][BM][BK]
    uint16_t* Bs = reinterpret_cast<uint16_t*>(smem + 2 * BM * BK * 2);  // [2][BN][BK]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int64_t mblk = blockIdx.x, nblk = blockIdx.y;
    const int64_t m0 = mblk * BM;

    // Per-thread staging coordinates: 4 chunks (16 B) of A and of B per K-tile.
    const uint16_t* a_src[4];
    const uint8_t* b_src[4];   // byte address of the row's chunk (bf16: 2 B / weight, fp8: 1)
    float b_sc[4];             // fp8 row scale
    int lds_off[4];
    constexpr int EB = WT ? 1 : 2;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int c = tid + 256 * i;       // chunk id 0..1023
        const int row = c >> 3, ch = c & 7;
        int64_t ar = m0 + row;
        if (ar >= p.M) ar = p.M - 1;
        a_src[i] = p.A + ar * p.lda + ch * 8;
        bool v;
        int64_t wr_row;
        const uint16_t* wbase = w_row<EPI>(p, nblk, row, v, EB, wr_row, b_sc[i]);
        b_src[i] = reinterpret_cast<const uint8_t*>(wbase) + ch * 8 * EB;
        lds_off[i] = row * BK + ((ch ^ (row & 7)) * 8);
    }

    const int nk = (int)((p.K + BK - 1) / BK);
    uint4 ra[4], rb[4];
    uint2 rq[4];
    // Unconditional loads at clamped addresses (chunks past K are re-reads of the last
    // chunk, zeroed by a select): a load under a condition is branched around and the
    // waitcnt pass then waits for everything at the join.
    auto gload = [&](int kt) {
        const int64_t kbase = (int64_t)kt * BK;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int ch = (tid + 256 * i) & 7;
            const bool ok = kbase + ch * 8 < p.K;
            const int64_t kb = ok ? kbase : p.K - 8 - ch * 8;
            ra[i] = *reinterpret_cast<const uint4*>(a_src[i] + kb);
            if constexpr (WT == 0) rb[i] = *reinterpret_cast<const uint4*>(b_src[i] + kb * 2);
            else rq[i] = *reinterpret_cast<const uint2*>(b_src[i] + kb);
            if (!ok) {
                ra[i] = make_uint4(0, 0, 0, 0);
                if constexpr (WT == 0) rb[i] = make_uint4(0, 0, 0, 0);
                else rq[i] = make_uint2(0, 0);
            }
        }
    };
    auto lstore = [&](int buf) {
        uint16_t* a = As + buf * BM * BK;
        uint16_t* b = Bs + buf * BN * BK;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            *reinterpret_cast<uint4*>(a + lds_off[i]) = ra[i];
            if constexpr (WT == 0) *reinterpret_cast<uint4*>(b + lds_off[i]) = rb[i];
            else *reinterpret_cast<uint4*>(b + lds_off[i]) = fp8x8_to_bf16(rq[i], b_sc[i]);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    gload(0);
    lstore(0);
    __syncthreads();

    const int fr = lane & 15, fq = lane >> 4;
    int cur = 0;
    for (int kt = 0; kt < nk; kt++) {
        if (kt + 1 < nk) gload(kt + 1);
        const uint16_t* a = As + cur * BM * BK;
        const uint16_t* b = Bs + cur * BN * BK;
#pragma unroll
        for (int ks = 0; ks < 2; ks++) {
            bf16x8 af[4], bfr[4];
            const int ch = ks * 4 + fq;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int row = wr * 64 + i * 16 + fr;
                af[i] = *reinterpret_cast<const bf16x8*>(a + row * BK + ((ch ^ (row & 7)) * 8));
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int row = wc * 64 + j * 16 + fr;
                bfr[j] = *reinterpret_cast<const bf16x8*>(b + row * BK + ((ch ^ (row & 7)) * 8));
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) lstore(cur ^ 1);
        __syncthreads();
        cur ^= 1;
    }

    // ---------------- epilogue.  C/D map: col = lane & 15, row = 4*(lane >> 4) + r.
    if constexpr (EPI == QIE_EPI_SWIGLU) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
#pragma unroll
            for (int jj = 0; jj < 2; jj++) {
                const int64_t col = nblk * 64 + 32 * wc + 16 * jj + fr;
                if (col >= p.N) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wr * 64 + i * 16 + fq * 4 + r;
                    if (row >= p.M) continue;
                    float g = rbf(acc[i][jj][r]);
                    float u = rbf(acc[i][jj + 2][r]);
                    float av = rbf(g * (1.0f / (1.0f + expf(-g))));
                    p.C[row * p.ldc + col] = f2bf(u * av);
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int64_t col = nblk * BN + wc * 64 + j * 16 + fr;
            if (col >= p.N) continue;
            float bias = 0.f;
            if constexpr (EPI == QIE_EPI_STORE) {
                const uint16_t* b = col < p.n0 ? p.b0 : (col < p.n01 ? p.b1 : p.b2);
                if (b) bias = bf2f(b[col < p.n0 ? col : (col < p.n01 ? col - p.n0 : col - p.n01)]);
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wr * 64 + i * 16 + fq * 4 + r;
                    if (row >= p.M) continue;
                    if constexpr (EPI == QIE_EPI_F32) {
                        reinterpret_cast<float*>(p.C)[row * p.ldc + col] = acc[i][j][r];
                        continue;
                    }
                    uint16_t* dst = p.C + row * p.ldc + col;
                    if constexpr (EPI == QIE_EPI_RESIDUAL)
                        *dst = f2bf(bf2f(*dst) + rbf(acc[i][j][r]));
                    else
                        *dst = f2bf(acc[i][j][r] + bias);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Large prefill GEMM (bf16 weights, K % 32 == 0, enough 256x256 tiles to fill the chip):
// 256x256 block tile, 8 waves as 2 (M) x 4 (N), 128x64 per wave = 8x4 accumulators of
// v_mfma_f32_16x16x32_bf16.  Both operands go global -> LDS by LDS-DMA
// (global_load_lds_dwordx4: one wave-instruction = 16 rows x 64 B, the LDS image
// lane-linear, the chunk swizzle applied to the SOURCE address) into a ring of four
// 32-deep k-tiles (4 x 32 KB): three k-tiles stay in flight across the raw s_barrier that
// opens each k-step and are retired by a counted vmcnt, never vmcnt(0) in the main loop
// (cdna_hip_programming.md §5 'Pipelining across barriers', 'What does break it').  One
// workgroup (2 waves per SIMD) per CU; the bijective XCD remap keeps the M tiles that
// share a weight tile on one XCD, so each weight tile comes from HBM into one L2 once.
namespace big {
constexpr int BM = 256, BK = 32, SLOTS = 4;
// slot = A rows then B rows, 64 B each: 32 KB at BN 256, 24 KB at BN 128
constexpr int slot_bytes(int bn) { return (BM + bn) * BK * 2; }
}  // namespace big

// chunk swizzle of 64-B LDS rows: the 16-B chunk c of row r sits at position c ^ swz(r).
// With it the 16 lanes of each ds_read_b128 lane group ({0-3,12-15,20-27}, ...) reading
// rows fr (and chunk g) of a 16-row fragment land on 16 distinct bank slots.
__device__ __forceinline__ int big_swz(int r) { return ((r >> 2) & 1) * 3; }

__device__ __forceinline__ void glds16(const void* src, void* lds) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

// weight row feeding tile column c (0..255) of column tile nt; SwiGLU tiles interleave
// 32 gate rows and the 32 up rows of the same outputs per 64-column wave slice
template <int EPI, int BNT>
__device__ __forceinline__ const uint16_t* big_wrow(const GemmParams& p, int64_t nt, int c) {
    if constexpr (EPI == QIE_EPI_SWIGLU) {
        constexpr int HALF = BNT / 8;   // gate (then up) rows per 1/4-tile wave slice
        const int ws = c / (BNT / 4), q = c % (BNT / 4);
        const int64_t j = nt * (BNT / 2) + ws * HALF + (q % HALF);
        const int64_t jj = j < p.N ? j : p.N - 1;
        return (q >= HALF ? p.w1 : p.w0) + jj * p.K;
    } else {
        const int64_t r = nt * BNT + c;
        const int64_t rr = r < p.N ? r : p.N - 1;
        if (rr < p.n0) return p.w0 + rr * p.K;
        if (rr < p.n01) return p.w1 + (rr - p.n0) * p.K;
        return p.w2 + (rr - p.n01) * p.K;
    }
}

template <int EPI, int BNT>
__global__ __launch_bounds__(512) void gemm_big_kernel(GemmParams p, int n_mt) {
#pragma clang fp contract(off)
    constexpr int TM = big::BM, TK = big::BK, NSL = big::SLOTS, SB = big::slot_bytes(BNT);
    constexpr int NJ = BNT / 64;            // 16-column fragments per wave (4 waves along N)
    constexpr int NBI = BNT / 128;          // B wave-instructions per k-tile per wave
    constexpr int LPK = 2 + NBI;            // LDS-DMA instructions per k-tile per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int fr = lane & 15, g = lane >> 4;
    // bijective XCD remap (cdna_hip_programming.md §5 'XCD swizzle must be bijective')
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
    const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int64_t mt = wid % n_mt, nt = wid / n_mt;
    const int64_t m0 = mt * TM;

    // staging: wave-instruction i (0, 1) of this wave moves rows [32 wave + 16 i, +16) of the
    // A tile and of the B tile; lane -> row (lane >> 2), LDS chunk (lane & 3)
    const uint16_t* asrc[2];
    const uint16_t* bsrc[NBI];
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int r = 32 * wave + 16 * i + (lane >> 2);
        const int c = (lane & 3) ^ big_swz(r);
        int64_t ar = m0 + r;
        ar = ar < p.M ? ar : p.M - 1;   // rows past M: re-read row M-1, never stored
        asrc[i] = p.A + ar * p.lda + c * 8;
    }
#pragma unroll
    for (int i = 0; i < NBI; i++) {
        const int r = 16 * NBI * wave + 16 * i + (lane >> 2);
        const int c = (lane & 3) ^ big_swz(r);
        bsrc[i] = big_wrow<EPI, BNT>(p, nt, r) + c * 8;
    }
    const int nk = (int)(p.K / TK);
    auto issue = [&](int kt) {
        unsigned char* slot = smem + (kt & (NSL - 1)) * SB;
        const int64_t k0 = (int64_t)kt * TK;
#pragma unroll
        for (int i = 0; i < 2; i++) glds16(asrc[i] + k0, slot + (32 * wave + 16 * i) * (TK * 2));
#pragma unroll
        for (int i = 0; i < NBI; i++) glds16(bsrc[i] + k0, slot + TM * TK * 2 + (16 * NBI * wave + 16 * i) * (TK * 2));
    };

    f32x4 acc[8][NJ];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < NJ; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue(0);
    if (nk > 1) issue(1);
    if (nk > 2) issue(2);
    for (int kt = 0; kt < nk; kt++) {
        // this wave's DMAs of tile kt have landed once at most the later tiles' are pending
        if (kt + 2 < nk) {
            if constexpr (LPK == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else if (kt + 1 < nk) {
            if constexpr (LPK == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();            // ... and every other wave's; slot kt-1 is free
        asm volatile("" ::: "memory");
        if (kt + 3 < nk) issue(kt + 3);          // into the slot of tile kt - 1
        const uint16_t* As = reinterpret_cast<const uint16_t*>(smem + (kt & (NSL - 1)) * SB);
        const uint16_t* Bs = As + TM * TK;
        bf16x8 af[8], bfr[NJ];
        // every fragment read is issued before the first MFMA (B first, then A in MFMA
        // order): one exposed LDS latency per k-tile instead of the compiler's four
        // read-two / wait-all / eight-MFMA batches (P = 2048: gate/up -2 %, O and down -6 %)
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const int row = wn * (BNT / 4) + j * 16 + fr;
            bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * TK + ((g ^ big_swz(row)) * 8));
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int row = wm * 128 + i * 16 + fr;
            af[i] = *reinterpret_cast<const bf16x8*>(As + row * TK + ((g ^ big_swz(row)) * 8));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < NJ; j++)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }

    // ---------------- epilogue.  C/D map: col = lane & 15, row = 4*(lane >> 4) + r.
    if constexpr (EPI == QIE_EPI_SWIGLU) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
#pragma unroll
            for (int jj = 0; jj < NJ / 2; jj++) {
                const int64_t col = nt * (BNT / 2) + (BNT / 8) * wn + 16 * jj + fr;
                if (col >= p.N) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    const float gg = rbf(acc[i][jj][r]);
                    const float uu = rbf(acc[i][jj + NJ / 2][r]);
                    const float av = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                    p.C[row * p.ldc + col] = f2bf(uu * av);
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const int64_t col = nt * BNT + wn * (BNT / 4) + j * 16 + fr;
            if (col >= p.N) continue;
            float bias = 0.f;
            if constexpr (EPI == QIE_EPI_STORE) {
                const uint16_t* b = col < p.n0 ? p.b0 : (col < p.n01 ? p.b1 : p.b2);
                if (b) bias = bf2f(b[col < p.n0 ? col : (col < p.n01 ? col - p.n0 : col - p.n01)]);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    if constexpr (EPI == QIE_EPI_F32) {
                        reinterpret_cast<float*>(p.C)[row * p.ldc + col] = acc[i][j][r];
                        continue;
                    }
                    uint16_t* dst = p.C + row * p.ldc + col;
                    if constexpr (EPI == QIE_EPI_RESIDUAL)
                        *dst = f2bf(bf2f(*dst) + rbf(acc[i][j][r]));
                    else
                        *dst = f2bf(acc[i][j][r] + bias);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Prefill GEMM, phase-interleaved (round 4; cdna_hip_programming.md §5 "The 256² 8-phase
// template", written for this NT layout).  256x256 block tile, BK = 64, 8 waves as 2 (M) x 4
// (N), 128x64 per wave = 8x4 accumulators; LDS = two 64-KB k-tile buffers (A rows then W
// rows, 128-B rows, 16-B chunk c of row r at c ^ ((r >> 1) & 7): conflict-free
// ds_read_b128 for the 16x16x32 fragments).  A k-tile is consumed in FOUR phases, one C
// quadrant (64 x 32 per wave, 16 MFMAs) each:
//   P1 (qa0, qb0) reads A[qa0] + B[qb0]    P2 (qa0, qb1) reads B[qb1]
//   P3 (qa1, qb1) reads A[qa1]             P4 (qa1, qb0) (B[qb0] kept in registers)
// and the k-tile is staged as four 16-KB units in the order it is read: UA0 (the qa0 A rows
// of both M halves), UB0, UB1, UA1 (2 LDS-DMA instructions per wave each).  Phase P3 of tile
// t stages UA0(t+2), P4 UB0(t+2), P1 of t+1 UB1(t+2), P2 of t+1 UA1(t+2): every unit lands in
// its buffer >= 2 phases after the last read of what it overwrites, and is read 5-6 phases
// after it was issued.  Each phase = [fragment reads, one unit's DMAs, the counted wait]
// s_barrier [lgkmcnt(0), 16 MFMAs] s_barrier; the wait is vmcnt(8) at the end of P4, P1,
// P2 (the unit read next phase has landed; 4 units stay in flight), never 0 before the
// last two tiles.  Waves 4-7 run one barrier behind waves 0-3 (an extra s_barrier before the
// loop, waves 0-3 one after it), so on every SIMD one wave's MFMAs overlap the other
// wave's reads and DMA issue.  Accumulation order per output = k order (as gemm_big).
typedef unsigned int u32x4_g8 __attribute__((ext_vector_type(4)));
namespace g8 {
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int BUF = (BM + BN) * BK * 2;   // 64 KB: A rows [0, 256) then W rows, 128 B each
}  // namespace g8

__device__ __forceinline__ int g8_swz(int r) { return (r >> 1) & 7; }

// Split-K (tiles < CUs: Qwen2-7B O / down at 2,048 rows have 112 256x256 tiles, QKV 144): the
// k-tiles of a tile are cut into `splitk` consecutive parts, one workgroup each (the remap
// keeps a tile's parts on one XCD).  Every part stores its fp32 accumulators write-through
// (sc1) into its slab [tile][part] (256 KB, each lane's 16-B accumulator quads in fragment
// order), drains, and adds to the tile's ticket; the part whose add comes last sums the slabs
// in PART order (sc1 loads: cdna_hip_programming.md §5 'Projection GEMM' item 2), so the result
// does not depend on arrival order, runs the epilogue and resets the ticket.
struct G8Split {
    int splitk;
    float* slab;       // [tiles][splitk][256 * 256] fp32
    unsigned* cnt;     // [tiles], zero at rest
};

template <int EPI>
__global__ __launch_bounds__(512) void gemm8_kernel(GemmParams p, int n_mt, G8Split sk) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int fr = lane & 15, g = lane >> 4;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
    const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int tile = wid / sk.splitk, part = wid % sk.splitk;
    const int64_t mt = tile % n_mt, nt = tile / n_mt;
    const int64_t m0 = mt * g8::BM;

    // DMA sources: unit u (0 UA0, 1 UB0, 2 UB1, 3 UA1), instruction i of this wave moves the
    // 8-row block b = 2 wave + i of the unit; lane -> row + (lane >> 3), LDS chunk lane & 7
    // (holding source chunk (lane & 7) ^ swz(row))
    const uint16_t* src[4][2];
    int dst_row[4][2];   // tile row of the block (A: 0..255, W: 0..255), wave-uniform
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int b = 2 * wave + i;
            int row0;
            if (u == 0 || u == 3) row0 = (b < 8 ? 8 * b : 128 + 8 * (b - 8)) + (u == 3 ? 64 : 0);
            else row0 = 64 * (b >> 2) + 8 * (b & 3) + (u == 2 ? 32 : 0);
            dst_row[u][i] = row0;
            const int r = row0 + (lane >> 3);
            const int cs = (lane & 7) ^ g8_swz(r);
            if (u == 0 || u == 3) {
                int64_t ar = m0 + r;
                ar = ar < p.M ? ar : p.M - 1;   // rows past M: re-read row M-1, never stored
                src[u][i] = p.A + ar * p.lda + cs * 8;
            } else {
                src[u][i] = big_wrow<EPI, 256>(p, nt, r) + cs * 8;
            }
        }
    const int nk_all = (int)(p.K / g8::BK);
    const int kb = (int)((int64_t)part * nk_all / sk.splitk);        // this part's k-tiles [kb, kb + nk)
    const int nk = (int)((int64_t)(part + 1) * nk_all / sk.splitk) - kb;
    auto stage = [&](int u, int kt) {   // unit u of local k-tile kt into buffer kt & 1
        unsigned char* buf = smem + (kt & 1) * g8::BUF + ((u == 0 || u == 3) ? 0 : g8::BM * 128);
        const int64_t k0 = (int64_t)(kb + kt) * g8::BK;
#pragma unroll
        for (int i = 0; i < 2; i++) glds16(src[u][i] + k0, buf + dst_row[u][i] * 128);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[4][2], fb0[2][2], fb1[2][2];

    auto read_a = [&](const unsigned char* buf, int qa) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int row = 128 * wm + 64 * qa + 16 * i + fr;
                fa[i][s2] = *reinterpret_cast<const bf16x8*>(buf + row * 128 + (((4 * s2 + g) ^ g8_swz(row)) * 16));
            }
    };
    auto read_b = [&](const unsigned char* buf, int qb, bf16x8 (&fb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int row = 64 * wn + 32 * qb + 16 * j + fr;
                fb[j][s2] = *reinterpret_cast<const bf16x8*>(buf + g8::BM * 128 + row * 128 +
                                                             (((4 * s2 + g) ^ g8_swz(row)) * 16));
            }
    };
    auto mfma_q = [&](int qa, int qb, const bf16x8 (&fb)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[4 * qa + i][2 * qb + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s2], fb[j][s2], acc[4 * qa + i][2 * qb + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto wait8 = [&](bool tail) {
        if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    };

    // prologue: UA0(0) UB0(0) UB1(0) UA1(0) UA0(1) UB0(1); P1(0) reads UA0(0), UB0(0)
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
    stage(0, 1); stage(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    bar();
    if (wm == 1) bar();   // waves 4-7 one barrier behind
    for (int t = 0; t < nk; t++) {
        const unsigned char* buf = smem + (t & 1) * g8::BUF;
        const bool tail = t >= nk - 2;
        // ---- P1 (qa0, qb0): reads A[qa0], B[qb0]; stages UB1(t+1); retires UB1(t)
        read_b(buf, 0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        read_a(buf, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) stage(2, t + 1);
        wait8(tail);
        bar();
        mfma_q(0, 0, fb0);
        bar();
        // ---- P2 (qa0, qb1): reads B[qb1]; stages UA1(t+1); retires UA1(t)
        read_b(buf, 1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) stage(3, t + 1);
        wait8(tail);
        bar();
        mfma_q(0, 1, fb1);
        bar();
        // ---- P3 (qa1, qb1): reads A[qa1]; stages UA0(t+2)
        read_a(buf, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 2 < nk) stage(0, t + 2);
        bar();
        mfma_q(1, 1, fb1);
        bar();
        // ---- P4 (qa1, qb0): B[qb0] from registers; stages UB0(t+2); retires UA0/UB0(t+1)
        if (t + 2 < nk) stage(1, t + 2);
        wait8(tail);
        bar();
        mfma_q(1, 0, fb0);
        bar();
    }
    if (wm == 0) bar();   // balance the barrier count of the two wave groups

    if (sk.splitk > 1) {   // uniform
        // this wave's quads: slab float offset ((wave * 32 + i * 4 + j) * 64 + lane) * 4
        const int64_t tb = (int64_t)tile * sk.splitk;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(sk.slab + (tb + part) * 65536, (short)0, 65536 * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g8, acc[i][j]), rs,
                                                       ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem);   // the staging array is free (one LDS object)
        if (tid == 0) {
            const unsigned old = __hip_atomic_fetch_add(sk.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = old == (unsigned)sk.splitk - 1 ? 1 : 0;
        }
        __syncthreads();
        if (*flag == 0) return;   // uniform
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < sk.splitk; q++) {   // part order: independent of who arrived last
            const auto rq = __builtin_amdgcn_make_buffer_rsrc(sk.slab + (tb + q) * 65536, (short)0, 65536 * 4, 0x00020000);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                  rq, ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16));
                    acc[i][j] = q == 0 ? v : acc[i][j] + v;
                }
        }
        if (tid == 0) __hip_atomic_store(sk.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---------------- epilogue (as gemm_big_kernel at BNT = 256)
    constexpr int NJ = 4;
    if constexpr (EPI == QIE_EPI_SWIGLU) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
#pragma unroll
            for (int jj = 0; jj < NJ / 2; jj++) {
                const int64_t col = nt * 128 + 32 * wn + 16 * jj + fr;
                if (col >= p.N) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    const float gg = rbf(acc[i][jj][r]);
                    const float uu = rbf(acc[i][jj + NJ / 2][r]);
                    const float av = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                    p.C[row * p.ldc + col] = f2bf(uu * av);
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const int64_t col = nt * 256 + wn * 64 + j * 16 + fr;
            if (col >= p.N) continue;
            float bias = 0.f;
            if constexpr (EPI == QIE_EPI_STORE) {
                const uint16_t* b = col < p.n0 ? p.b0 : (col < p.n01 ? p.b1 : p.b2);
                if (b) bias = bf2f(b[col < p.n0 ? col : (col < p.n01 ? col - p.n0 : col - p.n01)]);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    if constexpr (EPI == QIE_EPI_F32) {
                        reinterpret_cast<float*>(p.C)[row * p.ldc + col] = acc[i][j][r];
                        continue;
                    }
                    uint16_t* dst = p.C + row * p.ldc + col;
                    if constexpr (EPI == QIE_EPI_RESIDUAL)
                        *dst = f2bf(bf2f(*dst) + rbf(acc[i][j][r]));
                    else
                        *dst = f2bf(acc[i][j][r] + bias);
                }
            }
        }
    }
}

// Stream-K form of gemm8 (one workgroup per CU, a fixed grid).  Tile quantisation costs the
// one-tile-per-workgroup kernel whole rounds: gate/up at 2,048 rows has 1,184 tiles = 4.625
// rounds of 256 (the fifth round 62 % busy), QKV 144 tiles (one round, 56 % busy), down 112
// (split-K 2: 224 of 256 CUs).  Here the work is (tile, k-tile) units: the first
// dp_rounds * grid tiles go whole, one per workgroup per round; the k-tile units of the
// remaining tiles are cut into `grid` contiguous ranges of `chunk` units (tile-major, so a
// range is a tail of one tile, whole tiles, the head of another).  A tile covered by one
// range is finished in place; a tile shared by several ranges (its SEGMENTS) is finished by
// the last-arriving segment (ticket), which sums every segment's fp32 slab in SEGMENT order
// (k order; independent of arrival order) and runs the epilogue.  A workgroup's only
// partial segments are its range's first and last: slab [workgroup][first / last].
struct G8Stream {
    int dp_rounds;     // whole-tile rounds: tile r * grid + w for r < dp_rounds
    int tiles;         // all tiles; stream-K covers [dp_rounds * grid, tiles)
    int chunk;         // k-tile units per stream-K range
    float* slab;       // [grid][2][256 * 256] fp32
    unsigned* cnt;     // [tiles], zero at rest
};

template <int EPI>
__global__ __launch_bounds__(512) void gemm8sk_kernel(GemmParams p, int n_mt, G8Stream sk) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int fr = lane & 15, g = lane >> 4;
    const int nwg = gridDim.x, orig = blockIdx.x;
    // XCD-major workgroup index: consecutive indices (consecutive tiles, which share a weight
    // tile) sit on one XCD's L2
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
    const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int nk_all = (int)(p.K / g8::BK);

    int64_t m0 = 0, nt = 0;
    const uint16_t* src[4][2];
    int dst_row[4][2];
    auto set_tile = [&](int tile) {
        const int64_t mt = tile % n_mt;
        nt = tile / n_mt;
        m0 = mt * g8::BM;
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int b = 2 * wave + i;
                int row0;
                if (u == 0 || u == 3) row0 = (b < 8 ? 8 * b : 128 + 8 * (b - 8)) + (u == 3 ? 64 : 0);
                else row0 = 64 * (b >> 2) + 8 * (b & 3) + (u == 2 ? 32 : 0);
                dst_row[u][i] = row0;
                const int r = row0 + (lane >> 3);
                const int cs = (lane & 7) ^ g8_swz(r);
                if (u == 0 || u == 3) {
                    int64_t ar = m0 + r;
                    ar = ar < p.M ? ar : p.M - 1;
                    src[u][i] = p.A + ar * p.lda + cs * 8;
                } else {
                    src[u][i] = big_wrow<EPI, 256>(p, nt, r) + cs * 8;
                }
            }
    };
    int kb = 0;
    auto stage = [&](int u, int kt) {
        unsigned char* buf = smem + (kt & 1) * g8::BUF + ((u == 0 || u == 3) ? 0 : g8::BM * 128);
        const int64_t k0 = (int64_t)(kb + kt) * g8::BK;
#pragma unroll
        for (int i = 0; i < 2; i++) glds16(src[u][i] + k0, buf + dst_row[u][i] * 128);
    };

    f32x4 acc[8][4];
    bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
    auto read_a = [&](const unsigned char* buf, int qa) {
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int row = 128 * wm + 64 * qa + 16 * i + fr;
                fa[i][s2] = *reinterpret_cast<const bf16x8*>(buf + row * 128 + (((4 * s2 + g) ^ g8_swz(row)) * 16));
            }
    };
    auto read_b = [&](const unsigned char* buf, int qb, bf16x8 (&fb)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int row = 64 * wn + 32 * qb + 16 * j + fr;
                fb[j][s2] = *reinterpret_cast<const bf16x8*>(buf + g8::BM * 128 + row * 128 +
                                                             (((4 * s2 + g) ^ g8_swz(row)) * 16));
            }
    };
    auto mfma_q = [&](int qa, int qb, const bf16x8 (&fb)[2][2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    acc[4 * qa + i][2 * qb + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s2], fb[j][s2], acc[4 * qa + i][2 * qb + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto wait8 = [&](bool tail) {
        if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    };

    // k-tiles [kb_, kb_ + nk) of the current tile into acc (gemm8_kernel's main loop)
    auto run = [&](int kb_, int nk) {
        kb = kb_;
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
        if (nk > 1) {   // uniform
            stage(0, 1); stage(1, 1);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        if (wm == 1) bar();
        for (int t = 0; t < nk; t++) {
            const unsigned char* buf = smem + (t & 1) * g8::BUF;
            const bool tail = t >= nk - 2;
            read_b(buf, 0, fb0);
            __builtin_amdgcn_sched_barrier(0);
            read_a(buf, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 < nk) stage(2, t + 1);
            wait8(tail);
            bar();
            mfma_q(0, 0, fb0);
            bar();
            read_b(buf, 1, fb1);
            __builtin_amdgcn_sched_barrier(0);
            if (t + 1 < nk) stage(3, t + 1);
            wait8(tail);
            bar();
            mfma_q(0, 1, fb1);
            bar();
            read_a(buf, 1);
            __builtin_amdgcn_sched_barrier(0);
            if (t + 2 < nk) stage(0, t + 2);
            bar();
            mfma_q(1, 1, fb1);
            bar();
            if (t + 2 < nk) stage(1, t + 2);
            wait8(tail);
            bar();
            mfma_q(1, 0, fb0);
            bar();
        }
        if (wm == 0) bar();
    };

    auto epilogue = [&]() {
        constexpr int NJ = 4;
        if constexpr (EPI == QIE_EPI_SWIGLU) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
#pragma unroll
                for (int jj = 0; jj < NJ / 2; jj++) {
                    const int64_t col = nt * 128 + 32 * wn + 16 * jj + fr;
                    if (col >= p.N) continue;
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                        if (row >= p.M) continue;
                        const float gg = rbf(acc[i][jj][r]);
                        const float uu = rbf(acc[i][jj + NJ / 2][r]);
                        const float av = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                        p.C[row * p.ldc + col] = f2bf(uu * av);
                    }
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                const int64_t col = nt * 256 + wn * 64 + j * 16 + fr;
                if (col >= p.N) continue;
                float bias = 0.f;
                if constexpr (EPI == QIE_EPI_STORE) {
                    const uint16_t* b = col < p.n0 ? p.b0 : (col < p.n01 ? p.b1 : p.b2);
                    if (b) bias = bf2f(b[col < p.n0 ? col : (col < p.n01 ? col - p.n0 : col - p.n01)]);
                }
#pragma unroll
                for (int i = 0; i < 8; i++) {
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                        if (row >= p.M) continue;
                        if constexpr (EPI == QIE_EPI_F32) {
                            reinterpret_cast<float*>(p.C)[row * p.ldc + col] = acc[i][j][r];
                            continue;
                        }
                        uint16_t* dst = p.C + row * p.ldc + col;
                        if constexpr (EPI == QIE_EPI_RESIDUAL)
                            *dst = f2bf(bf2f(*dst) + rbf(acc[i][j][r]));
                        else
                            *dst = f2bf(acc[i][j][r] + bias);
                    }
                }
            }
        }
    };

    // ---- whole tiles
    for (int r = 0; r < sk.dp_rounds; r++) {
        set_tile(r * nwg + wid);
        run(0, nk_all);
        epilogue();
        __syncthreads();   // the next tile's DMA reuses the buffers
    }
    // ---- stream-K ranges
    const int64_t base = (int64_t)sk.dp_rounds * nwg * nk_all;
    const int64_t total = (int64_t)sk.tiles * nk_all;
    const int64_t ustart = base + (int64_t)wid * sk.chunk;
    const int64_t uend = ustart + sk.chunk < total ? ustart + sk.chunk : total;
    for (int64_t u = ustart; u < uend;) {   // uniform
        const int tile = (int)(u / nk_all);
        const int k0 = (int)(u % nk_all);
        const int k1 = (int)(uend - u < (int64_t)(nk_all - k0) ? k0 + (uend - u) : nk_all);
        set_tile(tile);
        run(k0, k1 - k0);
        bool emit = true;
        if (k0 != 0 || k1 != nk_all) {   // uniform: a shared tile
            const int slot = u == ustart ? 0 : 1;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(sk.slab + ((int64_t)wid * 2 + slot) * 65536, (short)0,
                                                              65536 * 4, 0x00020000);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g8, acc[i][j]), rs,
                                                           ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
            __syncthreads();
            // the tile's segments: ranges wf..wl
            const int64_t tu0 = (int64_t)tile * nk_all - base;
            const int wf = (int)(tu0 / sk.chunk), wl = (int)((tu0 + nk_all - 1) / sk.chunk);
            int* flag = reinterpret_cast<int*>(smem);
            if (tid == 0) {
                const unsigned old = __hip_atomic_fetch_add(sk.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                *flag = old == (unsigned)(wl - wf) ? 1 : 0;
            }
            __syncthreads();
            emit = *flag != 0;
            if (emit) {
                for (int w2 = wf; w2 <= wl; w2++) {   // segment (k) order
                    const int64_t s2 = base + (int64_t)w2 * sk.chunk;
                    const int slot2 = s2 / nk_all == tile ? 0 : 1;
                    const auto rq = __builtin_amdgcn_make_buffer_rsrc(sk.slab + ((int64_t)w2 * 2 + slot2) * 65536,
                                                                      (short)0, 65536 * 4, 0x00020000);
#pragma unroll
                    for (int i = 0; i < 8; i++)
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                          rq, ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16));
                            acc[i][j] = w2 == wf ? v : acc[i][j] + v;
                        }
                }
                if (tid == 0) __hip_atomic_store(sk.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (emit) epilogue();
        u += k1 - k0;
        __syncthreads();
    }
}

template <int EPI>
static int launch_gemm8_t(const GemmParams& p, int n_mt, int n_tiles, const G8Split& sk, hipStream_t st) {
    const void* fn = (const void*)gemm8_kernel<EPI>;
    constexpr size_t shm = 2 * (size_t)g8::BUF;
    static bool raised = false;
    if (!raised) {
        QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        raised = true;
    }
    hipLaunchKernelGGL((gemm8_kernel<EPI>), dim3((unsigned)(n_tiles * sk.splitk)), dim3(512), shm, st, p, n_mt, sk);
    QIE_LAUNCH_CHECK();
    return 0;
}
static int launch_gemm8(int epi, const GemmParams& p, int n_mt, int n_tiles, const G8Split& sk, hipStream_t st) {
    if (epi == QIE_EPI_SWIGLU) return launch_gemm8_t<QIE_EPI_SWIGLU>(p, n_mt, n_tiles, sk, st);
    if (epi == QIE_EPI_RESIDUAL) return launch_gemm8_t<QIE_EPI_RESIDUAL>(p, n_mt, n_tiles, sk, st);
    if (epi == QIE_EPI_F32) return launch_gemm8_t<QIE_EPI_F32>(p, n_mt, n_tiles, sk, st);
    return launch_gemm8_t<QIE_EPI_STORE>(p, n_mt, n_tiles, sk, st);
}

// Split-K slabs + tickets, one set per stream (streams of one device may run GEMMs at the same
// time: tensor-parallel ranks on one GPU in the tests), grown on demand outside graph capture.
struct G8Ws {
    float* slab = nullptr;
    unsigned* cnt = nullptr;
    size_t slab_bytes = 0, cnt_n = 0;
};
static std::mutex g8_mu;
static std::map<hipStream_t, G8Ws> g8_ws;

static int g8_workspace(hipStream_t st, int slabs, int tiles, G8Split* out) {
    std::lock_guard<std::mutex> lk(g8_mu);
    G8Ws& w = g8_ws[st];
    const size_t need = (size_t)slabs * 65536 * 4;
    if (need > w.slab_bytes || (size_t)tiles > w.cnt_n) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 1;   // no split
        QIE_HIP(hipStreamSynchronize(st));
        const size_t sb = std::max(need, w.slab_bytes), cn = std::max((size_t)tiles, w.cnt_n);   // never shrink
        if (w.slab) hipFree(w.slab);
        if (w.cnt) hipFree(w.cnt);
        w = G8Ws{};
        QIE_HIP(hipMalloc((void**)&w.slab, sb));
        QIE_HIP(hipMalloc((void**)&w.cnt, cn * 4));
        QIE_HIP(hipMemsetAsync(w.cnt, 0, cn * 4, st));   // ordered before this stream's GEMMs
        w.slab_bytes = sb;
        w.cnt_n = cn;
    }
    out->slab = w.slab;
    out->cnt = w.cnt;
    return 0;
}

template <int EPI>
static int launch_gemm8sk_t(const GemmParams& p, int n_mt, int grid, const G8Stream& sk, hipStream_t st) {
    const void* fn = (const void*)gemm8sk_kernel<EPI>;
    constexpr size_t shm = 2 * (size_t)g8::BUF;
    static bool raised = false;
    if (!raised) {
        QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        raised = true;
    }
    hipLaunchKernelGGL((gemm8sk_kernel<EPI>), dim3((unsigned)grid), dim3(512), shm, st, p, n_mt, sk);
    QIE_LAUNCH_CHECK();
    return 0;
}

// Stream-K plan + workspace (the split-K one: slab [grid][2] tiles, tickets [tiles]);
// *launched = false: a workspace would have to grow during a graph capture
static int launch_gemm8sk(int epi, const GemmParams& p, int n_mt, int tiles, hipStream_t st, bool* launched) {
    *launched = false;
    const int gk = dev_env("QIE_GEMM8_SK_GRID", 0);   // dev A/B: workgroups (default one per CU)
    const int grid = gk > 0 ? gk : (int)device_cu_count();
    const int nk = (int)(p.K / g8::BK);
    G8Stream sk;
    sk.tiles = tiles;
    sk.dp_rounds = tiles / grid;
    const int64_t rest = (int64_t)(tiles - sk.dp_rounds * grid) * nk;
    sk.chunk = (int)std::max<int64_t>(1, (rest + grid - 1) / grid);
    G8Split ws{1, nullptr, nullptr};
    if (rest > 0 && g8_workspace(st, 2 * grid, tiles, &ws) != 0) return 0;
    sk.slab = ws.slab;
    sk.cnt = ws.cnt;
    *launched = true;
    if (epi == QIE_EPI_SWIGLU) return launch_gemm8sk_t<QIE_EPI_SWIGLU>(p, n_mt, grid, sk, st);
    if (epi == QIE_EPI_RESIDUAL) return launch_gemm8sk_t<QIE_EPI_RESIDUAL>(p, n_mt, grid, sk, st);
    if (epi == QIE_EPI_F32) return launch_gemm8sk_t<QIE_EPI_F32>(p, n_mt, grid, sk, st);
    return launch_gemm8sk_t<QIE_EPI_STORE>(p, n_mt, grid, sk, st);
}

// parts per tile: the fewest rounds of (tile, part) items over the CUs, in units of a tile
// (112 tiles: 2 parts = one round of half tiles; 144 tiles: 3 parts, two rounds of thirds)
// (short parts lose: QKV at 3 x 19 and O at 2 x 28 k-tiles measured 108 -> 112 and 71 -> 69 us,
// the last arriver's serial slab read and the per-part pipeline fill eat the gain; down at
// 2 x 148: 309 -> 247 us), so a part keeps >= 64 k-tiles
static int g8_splitk(int64_t tiles, int64_t cus, int nk) {
    int best = 1;
    double best_t = 1e30;
    // k-tiles per part at least QIE_GEMM8_SK_MINK (dev A/B; default 64: K >= 4,096 per part).
    // Round 5: split-K 2 for the O projection at P = 2,048 (112 tiles -> 224, K = 3,584) ran
    // 94-98 vs 84 µs for the 256x128 kernel; QKV at 3 parts 114 vs 89 — the slab round trip
    // costs more than the idle CUs at this K
    const int mink = std::max(4, dev_env("QIE_GEMM8_SK_MINK", 64));
    for (int s = 1; s <= 4 && nk / s >= mink; s++) {
        const double t = (double)((tiles * s + cus - 1) / cus) / s;
        if (t < best_t - 1e-9) {
            best_t = t;
            best = s;
        }
    }
    return best;
}

template <int EPI, int BNT>
static int launch_gemm_big_t(const GemmParams& p, int n_mt, int n_tiles, hipStream_t st) {
    const void* fn = (const void*)gemm_big_kernel<EPI, BNT>;
    constexpr size_t shm = (size_t)big::SLOTS * big::slot_bytes(BNT);
    static bool raised = false;
    if (!raised) {
        QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        raised = true;
    }
    hipLaunchKernelGGL((gemm_big_kernel<EPI, BNT>), dim3((unsigned)n_tiles), dim3(512), shm, st, p, n_mt);
    QIE_LAUNCH_CHECK();
    return 0;
}

template <int BNT>
static int launch_gemm_big(int epi, const GemmParams& p, int n_mt, int n_tiles, hipStream_t st) {
    if (epi == QIE_EPI_SWIGLU) return launch_gemm_big_t<QIE_EPI_SWIGLU, BNT>(p, n_mt, n_tiles, st);
    if (epi == QIE_EPI_RESIDUAL) return launch_gemm_big_t<QIE_EPI_RESIDUAL, BNT>(p, n_mt, n_tiles, st);
    if (epi == QIE_EPI_F32) return launch_gemm_big_t<QIE_EPI_F32, BNT>(p, n_mt, n_tiles, st);
    return launch_gemm_big_t<QIE_EPI_STORE, BNT>(p, n_mt, n_tiles, st);
}

template <int WT>
static int launch_gemm(int epi, unsigned gm, const GemmParams& p, size_t shm, hipStream_t st) {
    if (epi == QIE_EPI_SWIGLU) {
        hipLaunchKernelGGL((gemm_kernel<QIE_EPI_SWIGLU, WT>), dim3(gm, (unsigned)cdiv(p.N, 64)), dim3(256), shm, st, p);
    } else if (epi == QIE_EPI_RESIDUAL) {
        hipLaunchKernelGGL((gemm_kernel<QIE_EPI_RESIDUAL, WT>), dim3(gm, (unsigned)cdiv(p.N, BN)), dim3(256), shm, st,
                           p);
    } else if (epi == QIE_EPI_F32) {
        hipLaunchKernelGGL((gemm_kernel<QIE_EPI_F32, WT>), dim3(gm, (unsigned)cdiv(p.N, BN)), dim3(256), shm, st, p);
    } else {
        hipLaunchKernelGGL((gemm_kernel<QIE_EPI_STORE, WT>), dim3(gm, (unsigned)cdiv(p.N, BN)), dim3(256), shm, st, p);
    }
    QIE_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------------------
// Block-scaled fp8 prefill GEMM (round 5; BASELINE config 4's "CDNA4 fp8 MFMA", numerics flag
// QIE_LINEAR_ACT_FP8):  C[m, n] = sum_k (2^ea[m] qa[m, k]) (sw[n] qw[n, k])  with e4m3
// activation codes qa and per-row power-of-two exponents ea (qie_quantize_rows_fp8), e4m3
// weight codes qw with power-of-two row scales sw (the engine's fp8 arena, plain or 16-row
// tiled).  Both scales are row constants, so they enter v_mfma_scale_f32_16x16x128_f8f6f4 as
// its per-lane e8m0 operands (every lane of an A row / B column passes the same byte) and the
// accumulators come out scaled: the epilogues are gemm8's.  The product of two e4m3 values is
// exact; the instruction's K = 128 per step doubles the bf16 rate per clock (MI355X_MICROARCH
// "Matrix cores": twice the cycles of the bf16 16x16 form at 4x the K).
//   Structure = gemm8_kernel's (256x256 tile, 8 waves 2 x 4, four phases per k-tile, LDS-DMA
// units in read order, waves 4-7 one barrier behind): a k-tile is BK = 128 codes, i.e. the
// same 128-B LDS rows as gemm8's 64 bf16, so the buffers, unit schedule, swizzle and waits are
// unchanged; a fragment is 32 codes (chunks 2g, 2g + 1 of the row: k = 32 g + [0, 32), the
// 16x16x128 lane map) and a phase issues 8 MFMAs of twice the cycles instead of 16.
// Tiled weights (QIE_LINEAR_FP8_T16) are gathered straight from their 1-KiB blocks by the
// per-lane DMA addresses (chunk c of row r: block (r / 16, c / 4), bytes 16 ((r % 16) +
// 16 (c % 4))), so the decode layout is the prefill's too — no bf16 copy is read.
namespace mx {
constexpr int BK = 128;   // codes per k-tile row (128 B)
}

struct MxParams {
    const uint8_t* A;     // [M][lda] e4m3 codes
    int64_t lda;          // bytes
    const uint8_t* ea;    // [M] e8m0 row exponents
    const uint8_t* w[3];  // fp8 segments: codes, then fp32 row scales
    const uint16_t* b[3];
    int64_t rows[3];      // segment rows
    int64_t n0, n01;
    int64_t M, K, N;
    uint16_t* C;
    int64_t ldc;
};

// segment, row-in-segment of tile column c (0..255) of column tile nt (big_wrow's mapping)
template <int EPI>
__device__ __forceinline__ int mx_wrow(const MxParams& p, int64_t nt, int c, int64_t& r) {
    if constexpr (EPI == QIE_EPI_SWIGLU) {
        const int ws = c / 64, q = c % 64;
        const int64_t j = nt * 128 + ws * 32 + (q % 32);
        r = j < p.N ? j : p.N - 1;
        return q >= 32 ? 1 : 0;
    } else {
        int64_t rr = nt * 256 + c;
        rr = rr < p.N ? rr : p.N - 1;
        if (rr < p.n0) { r = rr; return 0; }
        if (rr < p.n01) { r = rr - p.n0; return 1; }
        r = rr - p.n01;
        return 2;
    }
}

typedef int i32x8_mx __attribute__((ext_vector_type(8)));

template <int EPI, bool T16>
__global__ __launch_bounds__(512) void gemm8mx_kernel(MxParams p, int n_mt, G8Split sk, int dbg) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2, wn = wave & 3;
    const int fr = lane & 15, g = lane >> 4;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
    const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
    const int tile = wid / sk.splitk, part = wid % sk.splitk;
    const int64_t mt = tile % n_mt, nt = tile / n_mt;
    const int64_t m0 = mt * g8::BM;
    const int64_t K = p.K;

    // e8m0 operands, packed 4 per register (byte i of sa_pk[qa]: A row 128 wm + 64 qa + 16 i +
    // fr; byte 2 qb + j of sb_pk: B tile column 64 wn + 32 qb + 16 j + fr -> the exponent of the
    // weight row's power-of-two scale): 3 VGPRs, the budget gemm8's 254 leaves
    uint32_t sa_pk[2] = {0u, 0u}, sb_pk = 0u;
#pragma unroll
    for (int q = 0; q < 8; q++) {
        int64_t ar = m0 + 128 * wm + 16 * q + fr;
        ar = ar < p.M ? ar : p.M - 1;
        sa_pk[q >> 2] |= (uint32_t)p.ea[ar] << (8 * (q & 3));
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int64_t r;
        const int sg = mx_wrow<EPI>(p, nt, 64 * wn + 16 * j + fr, r);
        const uint8_t* base = sg == 0 ? p.w[0] : (sg == 1 ? p.w[1] : p.w[2]);
        const int64_t rows = sg == 0 ? p.rows[0] : (sg == 1 ? p.rows[1] : p.rows[2]);
        const uint32_t bits = __float_as_uint(reinterpret_cast<const float*>(base + rows * K)[r]);
        sb_pk |= ((bits >> 23) & 0xffu) << (8 * j);
    }
    // the exponents are waited for here, once: an opaque register pin makes them values of
    // this point, so no wait for them is left inside the DMA-pipelined loop
    asm volatile("" : "+v"(sa_pk[0]), "+v"(sa_pk[1]), "+v"(sb_pk));

    // DMA sources (gemm8's units and rows): A as 32-bit row offsets from p.A (4 VGPRs), W as
    // pointers (segments may lie anywhere)
    uint32_t aoff[2][2];
    const uint8_t* wsrc[2][2];
    int dst_row[4][2];
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const int b = 2 * wave + i;
            int row0;
            if (u == 0 || u == 3) row0 = (b < 8 ? 8 * b : 128 + 8 * (b - 8)) + (u == 3 ? 64 : 0);
            else row0 = 64 * (b >> 2) + 8 * (b & 3) + (u == 2 ? 32 : 0);
            dst_row[u][i] = row0;
            const int rw = row0 + (lane >> 3);
            const int cs = (lane & 7) ^ g8_swz(rw);
            if (u == 0 || u == 3) {
                int64_t ar = m0 + rw;
                ar = ar < p.M ? ar : p.M - 1;   // rows past M: re-read row M-1, never stored
                aoff[u == 3][i] = (uint32_t)(ar * p.lda + cs * 16);
            } else {
                int64_t r;
                const int sg = mx_wrow<EPI>(p, nt, rw, r);
                const uint8_t* base = sg == 0 ? p.w[0] : (sg == 1 ? p.w[1] : p.w[2]);
                if constexpr (T16)
                    wsrc[u - 1][i] = base + (r >> 4) * 16 * K + (cs >> 2) * 1024 + 16 * ((r & 15) + 16 * (cs & 3));
                else
                    wsrc[u - 1][i] = base + r * K + cs * 16;
            }
        }
    constexpr int64_t WSTEP = T16 ? 2048 : mx::BK;   // weight bytes per k-tile
    const int nk_all = (int)(K / mx::BK);
    const int kb = (int)((int64_t)part * nk_all / sk.splitk);
    const int nk = (int)((int64_t)(part + 1) * nk_all / sk.splitk) - kb;
    auto stage = [&](int u, int kt) {
        unsigned char* buf = smem + (kt & 1) * g8::BUF + ((u == 0 || u == 3) ? 0 : g8::BM * 128);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            if (u == 0 || u == 3)
                glds16(p.A + (int64_t)(kb + kt) * mx::BK + aoff[u == 3][i], buf + dst_row[u][i] * 128);
            else
                glds16(wsrc[u - 1][i] + (int64_t)(kb + kt) * WSTEP, buf + dst_row[u][i] * 128);
        }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    i32x8_mx fa[4], fb0[2], fb1[2];

    auto frag = [&](const unsigned char* rowp, int row) -> i32x8_mx {
        const u32x4_g8 lo = *reinterpret_cast<const u32x4_g8*>(rowp + (((2 * g) ^ g8_swz(row)) * 16));
        const u32x4_g8 hi = *reinterpret_cast<const u32x4_g8*>(rowp + (((2 * g + 1) ^ g8_swz(row)) * 16));
        return i32x8_mx{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
    };
    auto read_a = [&](const unsigned char* buf, int qa) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int row = 128 * wm + 64 * qa + 16 * i + fr;
            fa[i] = frag(buf + row * 128, row);
        }
    };
    auto read_b = [&](const unsigned char* buf, int qb, i32x8_mx (&fb)[2]) {
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int row = 64 * wn + 32 * qb + 16 * j + fr;
            fb[j] = frag(buf + g8::BM * 128 + row * 128, row);
        }
    };
    auto mfma_q = [&](int qa, int qb, const i32x8_mx (&fb)[2]) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++)
            {
                acc[4 * qa + i][2 * qb + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    fa[i], fb[j], acc[4 * qa + i][2 * qb + j], 0, 0, 0, (int)((sa_pk[qa] >> (8 * i)) & 0xffu), 0,
                    (int)((sb_pk >> (8 * (2 * qb + j))) & 0xffu));
                if (QIE_DBG(dbg == 1)) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto wait8 = [&](bool tail) {
        if (tail) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    };

    // prologue (gemm8's): UA0(0) UB0(0) UB1(0) UA1(0) UA0(1) UB0(1)
    stage(0, 0); stage(1, 0); stage(2, 0); stage(3, 0);
    if (nk > 1) { stage(0, 1); stage(1, 1); }
    if (nk > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (wm == 1) bar();
    for (int t = 0; t < nk; t++) {
        const unsigned char* buf = smem + (t & 1) * g8::BUF;
        const bool tail = t >= nk - 2;
        // keep the packed exponents loop-variant: the byte extractions stay next to their
        // MFMAs instead of being hoisted into 12 registers live across the loop
        asm volatile("" : "+v"(sa_pk[0]), "+v"(sa_pk[1]), "+v"(sb_pk));
        read_b(buf, 0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        read_a(buf, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) stage(2, t + 1);
        wait8(tail);
        bar();
        mfma_q(0, 0, fb0);
        bar();
        read_b(buf, 1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 1 < nk) stage(3, t + 1);
        wait8(tail);
        bar();
        mfma_q(0, 1, fb1);
        bar();
        read_a(buf, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + 2 < nk) stage(0, t + 2);
        bar();
        mfma_q(1, 1, fb1);
        bar();
        if (t + 2 < nk) stage(1, t + 2);
        wait8(tail);
        bar();
        mfma_q(1, 0, fb0);
        bar();
    }
    if (wm == 0) bar();

    if (sk.splitk > 1) {   // uniform (gemm8's split-K hand-off, part order)
        const int64_t tb = (int64_t)tile * sk.splitk;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(sk.slab + (tb + part) * 65536, (short)0, 65536 * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_g8, acc[i][j]), rs,
                                                       ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem);
        if (tid == 0) {
            const unsigned old = __hip_atomic_fetch_add(sk.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = old == (unsigned)sk.splitk - 1 ? 1 : 0;
        }
        __syncthreads();
        if (*flag == 0) return;
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int q = 0; q < sk.splitk; q++) {
            const auto rq = __builtin_amdgcn_make_buffer_rsrc(sk.slab + (tb + q) * 65536, (short)0, 65536 * 4, 0x00020000);
#pragma unroll
            for (int i = 0; i < 8; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                  rq, ((wave * 32 + i * 4 + j) * 64 + lane) * 16, 0, 16));
                    acc[i][j] = q == 0 ? v : acc[i][j] + v;
                }
        }
        if (tid == 0) __hip_atomic_store(sk.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---------------- epilogue (gemm8_kernel's)
    constexpr int NJ = 4;
    if constexpr (EPI == QIE_EPI_SWIGLU) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
#pragma unroll
            for (int jj = 0; jj < NJ / 2; jj++) {
                const int64_t col = nt * 128 + 32 * wn + 16 * jj + fr;
                if (col >= p.N) continue;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    const float gg = rbf(acc[i][jj][r]);
                    const float uu = rbf(acc[i][jj + NJ / 2][r]);
                    const float av = rbf(gg * (1.0f / (1.0f + expf(-gg))));
                    p.C[row * p.ldc + col] = f2bf(uu * av);
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            const int64_t col = nt * 256 + wn * 64 + j * 16 + fr;
            if (col >= p.N) continue;
            float bias = 0.f;
            if constexpr (EPI == QIE_EPI_STORE) {
                const uint16_t* b = col < p.n0 ? p.b[0] : (col < p.n01 ? p.b[1] : p.b[2]);
                if (b) bias = bf2f(b[col < p.n0 ? col : (col < p.n01 ? col - p.n0 : col - p.n01)]);
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int64_t row = m0 + wm * 128 + i * 16 + g * 4 + r;
                    if (row >= p.M) continue;
                    if constexpr (EPI == QIE_EPI_F32) {
                        reinterpret_cast<float*>(p.C)[row * p.ldc + col] = acc[i][j][r];
                        continue;
                    }
                    uint16_t* dst = p.C + row * p.ldc + col;
                    if constexpr (EPI == QIE_EPI_RESIDUAL)
                        *dst = f2bf(bf2f(*dst) + rbf(acc[i][j][r]));
                    else
                        *dst = f2bf(acc[i][j][r] + bias);
                }
            }
        }
    }
}

template <int EPI, bool T16>
static int launch_gemm8mx_t(const MxParams& p, int n_mt, int n_tiles, const G8Split& sk, hipStream_t st) {
    const void* fn = (const void*)gemm8mx_kernel<EPI, T16>;
    constexpr size_t shm = 2 * (size_t)g8::BUF;
    static bool raised = false;
    if (!raised) {
        QIE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        raised = true;
    }
    static const int dbg = dev_env("QIE_MX_DBG", 0);
    hipLaunchKernelGGL((gemm8mx_kernel<EPI, T16>), dim3((unsigned)(n_tiles * sk.splitk)), dim3(512), shm, st, p, n_mt,
                       sk, dbg);
    QIE_LAUNCH_CHECK();
    return 0;
}
template <bool T16>
static int launch_gemm8mx(int epi, const MxParams& p, int n_mt, int n_tiles, const G8Split& sk, hipStream_t st) {
    if (epi == QIE_EPI_SWIGLU) return launch_gemm8mx_t<QIE_EPI_SWIGLU, T16>(p, n_mt, n_tiles, sk, st);
    if (epi == QIE_EPI_RESIDUAL) return launch_gemm8mx_t<QIE_EPI_RESIDUAL, T16>(p, n_mt, n_tiles, sk, st);
    if (epi == QIE_EPI_F32) return launch_gemm8mx_t<QIE_EPI_F32, T16>(p, n_mt, n_tiles, sk, st);
    return launch_gemm8mx_t<QIE_EPI_STORE, T16>(p, n_mt, n_tiles, sk, st);
}

// QIE_LINEAR_ACT_FP8 (qie_ops.h): every M, one 256x256 kernel; split-K where the tiles do not
// fill the chip once (the fewest rounds of (tile, part) items; parts of >= 8 k-tiles)
static int gemm_mx(const qie_linear_args* a, hipStream_t st) {
    const bool t16 = (a->flags & QIE_LINEAR_FP8_T16) != 0;
    QIE_REQUIRE((a->flags & QIE_LINEAR_FP8) && a->x_exps, "qie_linear: ACT_FP8 needs fp8 weights and x_exps");
    QIE_REQUIRE(a->K % mx::BK == 0 && a->ldx >= a->K && a->ldx % 16 == 0,
                "qie_linear: ACT_FP8 needs K %% 128 == 0 and ldx (bytes) %% 16 == 0");
    QIE_REQUIRE(a->norm_w == nullptr && a->argmax_keys == nullptr, "qie_linear: ACT_FP8 takes no fused norm / arg-max");
    // the kernel keeps A row offsets (row * lda + column) in 32 bits: refuse what would wrap
    // (e.g. 8 x 32k rows of the down projection's K = 18,944) instead of reading wrong rows
    QIE_REQUIRE(((int64_t)cdiv(a->M, 256) * 256) * a->ldx < ((int64_t)1 << 32),
                "qie_linear: ACT_FP8 with M (%lld) x ldx (%lld) >= 2^32 bytes of codes (split the rows)",
                (long long)a->M, (long long)a->ldx);
    if (t16)
        QIE_REQUIRE(a->epilogue == QIE_EPI_SWIGLU ? a->N % 16 == 0
                                                  : a->seg_rows[0] % 16 == 0 && a->seg_rows[1] % 16 == 0 &&
                                                        a->seg_rows[2] % 16 == 0,
                    "qie_linear: tiled fp8 segments must be whole 16-row tiles");
    MxParams p;
    p.A = (const uint8_t*)a->x;
    p.lda = a->ldx;
    p.ea = a->x_exps;
    for (int i = 0; i < 3; i++) {
        p.w[i] = (const uint8_t*)a->w[i];
        p.b[i] = (const uint16_t*)a->bias[i];
    }
    const bool sw = a->epilogue == QIE_EPI_SWIGLU;
    p.rows[0] = sw ? a->N : a->seg_rows[0];
    p.rows[1] = sw ? a->N : a->seg_rows[1];
    p.rows[2] = sw ? 0 : a->seg_rows[2];
    p.n0 = a->seg_rows[0];
    p.n01 = a->seg_rows[0] + a->seg_rows[1];
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.C = (uint16_t*)a->y;
    p.ldc = a->ldy;
    const int64_t cols = sw ? 2 * a->N : a->N;
    const int64_t n_mt = cdiv(a->M, g8::BM), tiles = n_mt * cdiv(cols, 256);
    const int64_t cus = device_cu_count();
    const int nk = (int)(a->K / mx::BK);
    G8Split sk{1, nullptr, nullptr};
    // split only below half the chip (r05, same box, 2,048 rows): O (112 tiles) 91.0 unsplit
    // vs 78.0 split 3, down (112) 307 vs 188; QKV (144 tiles) 69.4 unsplit vs 93.9 split 3
    if (2 * tiles <= cus) {
        int best = 1;
        double best_t = 1e30;
        const int smax = dev_env("QIE_MX_SPLITK_MAX", 4);
        for (int s = 1; s <= smax && nk / s >= 8; s++) {
            const double t = (double)((tiles * s + cus - 1) / cus) / s;
            if (t < best_t - 1e-9) {
                best_t = t;
                best = s;
            }
        }
        if (best > 1 && g8_workspace(st, (int)tiles * best, (int)tiles, &sk) == 0) sk.splitk = best;
    }
    return t16 ? launch_gemm8mx<true>(a->epilogue, p, (int)n_mt, (int)tiles, sk, st)
               : launch_gemm8mx<false>(a->epilogue, p, (int)n_mt, (int)tiles, sk, st);
}

int gemm(const qie_linear_args* a, hipStream_t st) {
    if (a->flags & QIE_LINEAR_ACT_FP8) return gemm_mx(a, st);
    QIE_REQUIRE(a->norm_w == nullptr, "qie_linear: fused RMSNorm is GEMV-only (M <= 8)");
    QIE_REQUIRE(a->argmax_keys == nullptr, "qie_linear: fused arg-max is GEMV-only (M <= 8)");
    GemmParams p;
    p.A = (const uint16_t*)a->x;
    p.lda = a->ldx;
    p.w0 = (const uint16_t*)a->w[0];
    p.w1 = (const uint16_t*)a->w[1];
    p.w2 = (const uint16_t*)a->w[2];
    p.b0 = (const uint16_t*)a->bias[0];
    p.b1 = (const uint16_t*)a->bias[1];
    p.b2 = (const uint16_t*)a->bias[2];
    p.n0 = a->seg_rows[0];
    p.n01 = a->seg_rows[0] + a->seg_rows[1];
    p.M = a->M;
    p.K = a->K;
    p.N = a->N;
    p.wrows = 0;
    p.C = (uint16_t*)a->y;
    p.ldc = a->ldy;
    const size_t shm = (size_t)2 * (BM + BN) * BK * 2;
    const unsigned gm = (unsigned)cdiv(a->M, BM);
    QIE_REQUIRE(a->K % 8 == 0, "qie_linear: GEMM needs K %% 8 == 0");
    if (!(a->flags & QIE_LINEAR_FP8) && a->K % big::BK == 0 && a->ldx % 8 == 0) {
        // LDS-DMA kernel: 256x256 tiles when they fill the chip at least once (config 4's
        // O / down at 8,192 rows: 448 tiles; the generic 128x128 kernel took them before), else
        // 256x128 when those fill >= 3/4 of it in one round (Qwen2-7B O and down projections
        // at 2,048 rows: 112 vs 224 tiles on 256 CUs), else 256x256 in one round (below).
        // args.flags QIE_LINEAR_TILE256 / TILE128 force a tile (tests; dev builds also
        // QIE_GEMM_BIG = 1 / 2, 0 disables the kernel for A/B timing).
        const int64_t cols = a->epilogue == QIE_EPI_SWIGLU ? 2 * a->N : a->N;
        const int64_t n_mt = cdiv(a->M, big::BM);
        const int64_t t256 = n_mt * cdiv(cols, 256), t128 = n_mt * cdiv(cols, 128);
        const int64_t cus = device_cu_count();
        const int force = (a->flags & QIE_LINEAR_TILE256) ? 1 : (a->flags & QIE_LINEAR_TILE128) ? 2
                                                                                            : dev_env("QIE_GEMM_BIG", -1);
        // phase-interleaved 256x256 kernel (K a multiple of 64, >= 4 k-tiles): Qwen2-7B gate/up at 2,048
        // rows 612 -> 488 us, bit-identical to gemm_big; down split-K 2: 309 -> 247 us
        const bool g8ok = a->K % g8::BK == 0 && a->K >= 4 * g8::BK;
        const int g8mode = dev_env("QIE_GEMM8", 2);   // 2 (default): + split-K below; 1: full-chip grids only; 0: off
        // stream-K (QIE_GEMM8 = 3; args.flags QIE_LINEAR_STREAMK): any tile count, one workgroup per CU
        if (g8ok && ((a->flags & QIE_LINEAR_STREAMK) || (g8mode == 3 && force < 0 && a->M >= big::BM))) {
            bool launched = false;
            const int rc = launch_gemm8sk(a->epilogue, p, (int)n_mt, (int)t256, st, &launched);
            if (rc || launched) return rc;
        }
        if (g8ok && g8mode != 0 && force != 2 && (force == 1 || (force < 0 && a->M >= big::BM && t256 >= cus))) {
            G8Split sk{1, nullptr, nullptr};
            return launch_gemm8(a->epilogue, p, (int)n_mt, (int)t256, sk, st);
        }
        if (g8ok && g8mode == 2 && force < 0 && a->M >= big::BM && t256 < cus) {
            const int s = g8_splitk(t256, cus, (int)(a->K / g8::BK));
            G8Split sk{1, nullptr, nullptr};
            // unsplit, 256x256 tiles must still cover half the chip: QKV at 144 tiles 101.7 ->
            // 87.8 us, but O at 112 tiles 78 -> 103 us (its 256x128 kernel fills 224 CUs)
            if ((s == 1 && 2 * t256 >= cus) || (s > 1 && g8_workspace(st, (int)t256 * s, (int)t256, &sk) == 0 && (sk.splitk = s) > 1))
                return launch_gemm8(a->epilogue, p, (int)n_mt, (int)t256, sk, st);
        }
        if (force == 1 || (force < 0 && a->M >= big::BM && t256 >= cus))
            return launch_gemm_big<256>(a->epilogue, p, (int)n_mt, (int)t256, st);
        if (force == 2 || (force < 0 && a->M >= big::BM && t128 >= (3 * cus) / 4 && t128 <= cus))
            return launch_gemm_big<128>(a->epilogue, p, (int)n_mt, (int)t128, st);
        // 256-column tiles in ONE round when 128-column ones would take two (Qwen2-7B QKV at
        // 2,048 rows: 144 vs 288 tiles on 256 CUs): 124 -> 99 us against the generic kernel
        if (force < 0 && a->M >= big::BM && t256 >= cus / 2 && t256 <= cus && t128 > cus)
            return launch_gemm_big<256>(a->epilogue, p, (int)n_mt, (int)t256, st);
    }
    if (a->flags & QIE_LINEAR_FP8) return launch_gemm<1>(a->epilogue, gm, p, shm, st);
    return launch_gemm<0>(a->epilogue, gm, p, shm, st);
}

}  // namespace qie
