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

int gemm(const qie_linear_args* a, hipStream_t st) {
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
