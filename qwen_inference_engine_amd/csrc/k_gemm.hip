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
    if (a->flags & QIE_LINEAR_FP8) return launch_gemm<1>(a->epilogue, gm, p, shm, st);
    return launch_gemm<0>(a->epilogue, gm, p, shm, st);
}

}  // namespace qie
