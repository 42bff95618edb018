// conv.hip — client-batched implicit-GEMM convolution / linear on fp32 MFMA (gfx950).
//
// Replaces nn.Conv2d / nn.Linear forward+backward of the reference models
// (src/shared/models_pytorch.py:59-246) as driven by LocalTrainer._train_epoch
// (src/shared/training.py:192-197).  All three products are one kernel
// template, one GEMM per client slot (grid.z), each client with its own
// weights (FedAvg clients never share parameters during local training):
//
//   FWD   : Y[co][pix]      = sum_{ci,kh,kw} W[co][ci,kh,kw] * im2col(X)[ci,kh,kw][pix]
//   DGRAD : dX[ci][pix_in]  = sum_{co,kh,kw} W[co][ci,kh,kw] * col(dY)[co,kh,kw][pix_in]
//   WGRAD : dW[co][ci,kh,kw]= sum_{pix}      dY[co][pix]     * im2col(X)[ci,kh,kw][pix]
//
// GEMM row index m sits in the MFMA accumulator REGISTERS and the column index
// n on the LANES, so the pixel dimension (contiguous in NCHW) is what 32
// consecutive lanes store: every epilogue store is a 128-B coalesced segment.
// Operands are staged global -> registers -> LDS (double buffered, one barrier
// per K-step) in k-major [BK][B{M,N}+1] images: a lane's MFMA operand read
// (32 consecutive m or n at one k) is bank-conflict free for ds_read_b32, and
// the +1 pad makes the k-fast staging writes conflict free too.
// v_mfma_f32_32x32x2_f32 (exact fp32, 64 cyc/SIMD) is the MAC engine; each
// wave owns an FM x FN grid of 32x32 accumulators.
#include "fh_common.h"
#include "splitbn.h"

#include <cstdlib>

namespace fh {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// OP_DGRAD_S2: DGRAD of a stride-2 convolution (3x3/p1 or 1x1/p0) split into the four
// output-pixel parity phases (ih % 2, iw % 2).  A phase's pixels receive only the taps whose
// (ih + pad - kh) is even: 1, 2, 2 and 4 of the 3x3 kernel's 9 (the 1x1 kernel: its one tap
// in phase (0,0), none elsewhere), so each phase is a dense implicit GEMM with
// K = cout * taps instead of the generic DGRAD's cout * 9 with 3 of every 4 terms zero.
enum { OP_FWD = 0, OP_DGRAD = 1, OP_WGRAD = 2, OP_DGRAD_S2 = 3 };

// Dropout fused into a FWD epilogue (F.dropout after the ReLU of a classifier layer,
// models_pytorch.py:153-163): element e of a client's output [img][cout][oh][ow] is kept with
// probability keep (Philox keyed by (seed + *seed_dev, client, e), dropout_fwd_kernel's draw)
// and scaled by 1/keep; mode 1 writes the keep-mask, mode 2 reads an injected one.
struct DropArgs {
    uint8_t* mask;
    int64_t m_cs;
    int mode;  // 0: off
    float keep, scale;
    uint64_t seed;
    const uint64_t* seed_dev;
};

// The Philox key of a client row (key = seed + *seed_dev, row = philox_row): read once per thread
// ahead of an element loop.  r05: read per element, every uint8 keep-mask store (which may alias
// anything) forced the compiler to reload the key words after it — three dependent global
// round trips per element in the classifier forward's epilogue (fc2: 18 us for 8 workgroups).
struct DropKey {
    uint64_t seed, row;
};
__device__ __forceinline__ DropKey drop_key(const DropArgs& d, int z) {
    DropKey k{0ull, 0ull};
    if (d.mode == 1) {
        k.seed = d.seed + (d.seed_dev ? *d.seed_dev : 0ull);
        k.row = philox_row(d.seed_dev, z);
    }
    return k;
}
__device__ __forceinline__ float apply_dropout(const DropArgs& d, const DropKey& k, int z,
                                               int64_t e, float v) {
    uint8_t keep;
    if (d.mode == 1) {
        const uint4 r = Philox::gen(k.seed, k.row, (uint64_t)e);
        keep = u01(r.x) <= d.keep ? 1 : 0;
        d.mask[z * d.m_cs + e] = keep;
    } else {
        keep = d.mask[z * d.m_cs + e];
    }
    return keep ? v * d.scale : 0.f;
}

struct ConvArgs {
    const float* x;     // FWD/WGRAD: input activations; DGRAD: unused
    const float* wt;    // FWD/DGRAD: weights
    const float* dy;    // DGRAD/WGRAD: output gradient
    const float* bias;  // FWD: bias or null
    float* out;         // FWD: y, DGRAD: dx, WGRAD: split-K partials
    int64_t x_cs, w_cs, dy_cs, b_cs, out_cs;
    const int32_t* counts;
    int batch, cin, h, w, cout, oh, ow, pad;
    int relu;
    int accumulate;      // DGRAD: dx += result
    int splits, kchunk;  // split-K (WGRAD always; FWD/DGRAD when the grid is small)
    float* bias_part;    // WGRAD: per-split conv-bias partial sums [z][split][M] (or null)
    float* sq_part;      // WGRAD per-sample mode: sum of squares of each tile -> [z][split][tile]
    int sq_bias;         //   ... including the conv-bias gradient (first n-tile)
    int M, N, K;         // GEMM extents at full batch
    FastDiv fd_ohw, fd_ow, fd_hw, fd_w;
    DropArgs drop;       // FWD: dropout after bias / ReLU (unsplit launches; else the epilogue)
    // OP_DGRAD_S2, nullable: the weights re-laid phase-major by pack_dgrad_s2_kernel —
    // [client][phase][ci][co * taps + t] — so the A tile loads run along k (the gather from
    // W[co][ci][kh][kw] touches one cache line per lane: address-bound)
    const float* wp;
    int64_t wp_cs;
};

// Taps of a stride-2 DGRAD phase before phase ph (3x3/p1: 1, 2, 2, 4; 1x1/p0: 1, 0, 0, 0)
__host__ __device__ constexpr int s2_tap_prefix(int kh, int ph) {
    return kh == 3 ? (ph == 0 ? 0 : ph == 1 ? 1 : ph == 2 ? 3 : 5) : (ph == 0 ? 0 : 1);
}

template <int OP, int KH, int KW, int S, int BM, int BN, int BK, int WAVES_M>
__global__ void __launch_bounds__(256) igemm_kernel(const ConvArgs a) {
    constexpr int WAVES_N = 4 / WAVES_M;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int FM = WM / 32, FN = WN / 32;
    constexpr int KHW = KH * KW;
    constexpr int NA = BM * BK / 256, NB = BN * BK / 256;
    static_assert(FM >= 1 && FN >= 1 && NA >= 1 && NB >= 1, "tile");
    static_assert((256 % BN) == 0 || OP == OP_WGRAD, "n-fast B mapping needs BN | 256");

    __shared__ float As[2][BK][BM + 1];
    __shared__ float Bs[2][BK][BN + 1];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WAVES_N, wn = wid % WAVES_N;

    // blockIdx.z = client * splits + split (split-K: WGRAD always, FWD/DGRAD on small grids);
    // OP_DGRAD_S2: (client * 4 + phase) * splits + split
    constexpr bool DG2 = (OP == OP_DGRAD_S2);
    const int zz = blockIdx.z / a.splits;
    const int split = blockIdx.z - zz * a.splits;
    const int z = DG2 ? (zz >> 2) : zz;
    const int py = DG2 ? ((zz >> 1) & 1) : 0, px = DG2 ? (zz & 1) : 0;
    // taps of this phase per dimension (3x3/p1: 1 even, 2 odd; 1x1/p0: 1 even, 0 odd)
    const int nth = KH == 3 ? 1 + py : 1 - py, ntw = KW == 3 ? 1 + px : 1 - px;
    const int lg_tw = ntw == 2, lg_t = (nth == 2) + lg_tw;
    const bool partial_out = (OP == OP_WGRAD) || a.splits > 1;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int ohw = a.oh * a.ow, hw = a.h * a.w;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

    // GEMM extents for this client (partial last batch shrinks the pixel dim).
    int M = a.M, N = a.N, kbeg = 0, kend = a.K;
    if constexpr (OP == OP_FWD || DG2) N = cnt * ohw;
    if constexpr (OP == OP_DGRAD) N = cnt * hw;
    if constexpr (OP == OP_WGRAD) {
        const int kv = cnt * ohw;
        kbeg = split * a.kchunk;
        kend = min(kv, kbeg + a.kchunk);
    } else {
        if (n0 >= N) return;
        kbeg = split * a.kchunk;
        kend = min(DG2 ? a.cout * nth * ntw : a.K, kbeg + a.kchunk);
    }

    // ---------------- per-thread fixed coordinates -----------------------
    // FWD / DGRAD: B is loaded n-fast; thread owns column nb = tid % BN.
    const int nb = tid % BN;
    bool bcol_ok = false;
    const float* bcol_base = nullptr;
    int bi0 = 0, bj0 = 0;  // FWD: ih0/iw0 of the output pixel; DGRAD: ih/iw of the input pixel
    if constexpr (OP == OP_FWD || OP == OP_DGRAD || DG2) {
        const int n = n0 + nb;
        bcol_ok = n < N;
        uint32_t img, p, r, c;
        if constexpr (DG2) {  // n = (img, oy', ox') of the phase grid -> dX pixel (2oy'+py, 2ox'+px)
            a.fd_ohw.divmod(bcol_ok ? n : 0, img, p);
            a.fd_ow.divmod(p, r, c);
            bi0 = 2 * (int)r + py;
            bj0 = 2 * (int)c + px;
            bcol_base = a.dy + z * a.dy_cs + (int64_t)img * a.cout * ohw;
        } else if constexpr (OP == OP_FWD) {
            a.fd_ohw.divmod(bcol_ok ? n : 0, img, p);
            a.fd_ow.divmod(p, r, c);
            bi0 = (int)r * S - a.pad;
            bj0 = (int)c * S - a.pad;
            bcol_base = a.x + z * a.x_cs + (int64_t)img * a.cin * hw;
        } else {
            a.fd_hw.divmod(bcol_ok ? n : 0, img, p);
            a.fd_w.divmod(p, r, c);
            bi0 = (int)r + a.pad;
            bj0 = (int)c + a.pad;
            bcol_base = a.dy + z * a.dy_cs + (int64_t)img * a.cout * ohw;
        }
    }
    const float* wz = nullptr;
    if constexpr (OP != OP_WGRAD) wz = a.wt + z * a.w_cs;
    const float* wpz = nullptr;  // this (client, phase)'s packed weights [ci][co * taps]
    if constexpr (DG2)
        if (a.wp) wpz = a.wp + z * a.wp_cs + (int64_t)s2_tap_prefix(KH, 2 * py + px) * a.cin * a.cout;

    float ra[NA], rb[NB];

    auto load_tiles = [&](int k0) {
        if constexpr (OP == OP_FWD) {
            // A[m][k] = W[m][k], k-fast.
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int e = tid + i * 256, mm = e / BK, kk = e % BK;
                const int m = m0 + mm, k = k0 + kk;
                ra[i] = (m < M && k < kend) ? wz[(int64_t)m * a.K + k] : 0.f;
            }
            // B[k][n] = X[img][ci][ih0+kh][iw0+kw], n-fast.
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int e = tid + i * 256, kk = e / BN;
                const int k = k0 + kk;
                const int ci = k / KHW, rr = k - ci * KHW;
                const int kh = rr / KW, kw = rr - kh * KW;
                const int ih = bi0 + kh, iw = bj0 + kw;
                const bool ok = bcol_ok && k < kend && (unsigned)ih < (unsigned)a.h &&
                                (unsigned)iw < (unsigned)a.w;
                rb[i] = ok ? bcol_base[(int64_t)ci * hw + ih * a.w + iw] : 0.f;
            }
        } else if constexpr (DG2) {
            // k = (co, tap): tap -> (kh, kw) of this phase; odd phases take kh in {0, 2}
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int e = tid + i * 256, mm = e / BK, kk = e % BK;
                const int m = m0 + mm, k = k0 + kk;
                if (a.wp) {
                    ra[i] = (m < M && k < kend) ? wpz[(int64_t)m * (a.cout << lg_t) + k] : 0.f;
                    continue;
                }
                const int co = k >> lg_t, t = k & ((1 << lg_t) - 1);
                const int kh = KH == 3 ? (py ? 2 * (t >> lg_tw) : 1) : 0;
                const int kw = KW == 3 ? (px ? 2 * (t & ((1 << lg_tw) - 1)) : 1) : 0;
                ra[i] = (m < M && k < kend) ? wz[((int64_t)co * a.cin + m) * KHW + kh * KW + kw]
                                            : 0.f;
            }
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int e = tid + i * 256, kk = e / BN;
                const int k = k0 + kk;
                const int co = k >> lg_t, t = k & ((1 << lg_t) - 1);
                const int kh = KH == 3 ? (py ? 2 * (t >> lg_tw) : 1) : 0;
                const int kw = KW == 3 ? (px ? 2 * (t & ((1 << lg_tw) - 1)) : 1) : 0;
                const int oy = (bi0 + a.pad - kh) >> 1, ox = (bj0 + a.pad - kw) >> 1;  // exact
                const bool ok = bcol_ok && k < kend && (unsigned)oy < (unsigned)a.oh &&
                                (unsigned)ox < (unsigned)a.ow;
                rb[i] = ok ? bcol_base[(int64_t)co * ohw + oy * a.ow + ox] : 0.f;
            }
        } else if constexpr (OP == OP_DGRAD) {
            // A[m=ci][k=(co,kh,kw)] = W[co][ci][kh][kw], k-fast.
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int e = tid + i * 256, mm = e / BK, kk = e % BK;
                const int m = m0 + mm, k = k0 + kk;
                const int co = k / KHW, rr = k - co * KHW;
                ra[i] = (m < M && k < kend) ? wz[((int64_t)co * a.cin + m) * KHW + rr] : 0.f;
            }
            // B[k=(co,kh,kw)][n=(img,ih,iw)] = dY[img][co][oh][ow], oh*S = ih+pad-kh.
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int e = tid + i * 256, kk = e / BN;
                const int k = k0 + kk;
                const int co = k / KHW, rr = k - co * KHW;
                const int kh = rr / KW, kw = rr - kh * KW;
                int oy = bi0 - kh, ox = bj0 - kw;
                bool ok = bcol_ok && k < kend;
                if constexpr (S != 1) {
                    ok = ok && oy >= 0 && ox >= 0 && (oy % S) == 0 && (ox % S) == 0;
                    oy /= S;
                    ox /= S;
                }
                ok = ok && (unsigned)oy < (unsigned)a.oh && (unsigned)ox < (unsigned)a.ow;
                rb[i] = ok ? bcol_base[(int64_t)co * ohw + oy * a.ow + ox] : 0.f;
            }
        } else {
            // WGRAD: both operands k(=pixel)-fast; thread owns pixel kk = tid % BK.
            const int kk = tid % BK;
            const int k = k0 + kk;
            const bool kok = k < kend;
            uint32_t img, p, r, c;
            a.fd_ohw.divmod(kok ? k : 0, img, p);
            a.fd_ow.divmod(p, r, c);
            const float* dyb = a.dy + z * a.dy_cs + (int64_t)img * a.cout * ohw + p;
            const float* xb = a.x + z * a.x_cs + (int64_t)img * a.cin * hw;
            const int ih0 = (int)r * S - a.pad, iw0 = (int)c * S - a.pad;
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int m = m0 + (tid / BK) + i * (256 / BK);
                ra[i] = (kok && m < M) ? dyb[(int64_t)m * ohw] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int n = n0 + (tid / BK) + i * (256 / BK);
                const int ci = n / KHW, rr = n - ci * KHW;
                const int kh = rr / KW, kw = rr - kh * KW;
                const int ih = ih0 + kh, iw = iw0 + kw;
                const bool ok = kok && n < N && (unsigned)ih < (unsigned)a.h &&
                                (unsigned)iw < (unsigned)a.w;
                rb[i] = ok ? xb[(int64_t)ci * hw + ih * a.w + iw] : 0.f;
            }
        }
    };

    auto store_tiles = [&](int buf) {
        if constexpr (OP == OP_WGRAD) {
            const int kk = tid % BK;
#pragma unroll
            for (int i = 0; i < NA; ++i) As[buf][kk][(tid / BK) + i * (256 / BK)] = ra[i];
#pragma unroll
            for (int i = 0; i < NB; ++i) Bs[buf][kk][(tid / BK) + i * (256 / BK)] = rb[i];
        } else {
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int e = tid + i * 256;
                As[buf][e % BK][e / BK] = ra[i];
            }
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int e = tid + i * 256;
                Bs[buf][e / BN][e % BN] = rb[i];
            }
        }
    };

    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const bool do_bias = (OP == OP_WGRAD) && (a.bias_part != nullptr || a.sq_bias) &&
                         blockIdx.x == 0;
    float bsum = 0.f;
    if (kbeg < kend) {
        load_tiles(kbeg);
        store_tiles(0);
        __syncthreads();
        int buf = 0;
        const int kh_lane = lane >> 5, col = lane & 31;
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            const bool more = k0 + BK < kend;
            if (more) load_tiles(k0 + BK);
            if constexpr (OP == OP_WGRAD) {
                // conv bias gradient = row sums of A = dY over the pixel (k) range: folded in
                // here (first n-tile only) instead of a separate pass over dY.
                if (do_bias && tid < BM) {
#pragma unroll
                    for (int kk = 0; kk < BK; ++kk) bsum += As[buf][kk][tid];
                }
            }
#pragma unroll
            for (int kk = 0; kk < BK; kk += 2) {
                float av[FM], bv[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) av[i] = As[buf][kk + kh_lane][wm * WM + i * 32 + col];
#pragma unroll
                for (int j = 0; j < FN; ++j) bv[j] = Bs[buf][kk + kh_lane][wn * WN + j * 32 + col];
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
            }
            if (more) store_tiles(buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    }

    // ---------------- epilogue ------------------------------------------
    // per-sample squared norm (DP-SGD): one split per image; the tile's dW_i (and db_i)
    // are reduced to a sum of squares instead of being stored
    if constexpr (OP == OP_WGRAD) {
        if (a.sq_part) {
            __shared__ float sq_red[4];
            const int rb2 = 4 * (lane >> 5), c2 = lane & 31;
            float sq = 0.f;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + rb2;
                        const int n = n0 + wn * WN + j * 32 + c2;
                        if (m < M && n < N) sq += acc[i][j][r] * acc[i][j][r];
                    }
            if (a.sq_bias && blockIdx.x == 0 && tid < BM && m0 + tid < M) sq += bsum * bsum;
            sq = wave_sum(sq);
            if (lane == 0) sq_red[wid] = sq;
            __syncthreads();
            if (tid == 0)
                a.sq_part[(int64_t)blockIdx.z * gridDim.x * gridDim.y + blockIdx.y * gridDim.x +
                          blockIdx.x] = (sq_red[0] + sq_red[1]) + (sq_red[2] + sq_red[3]);
            return;
        }
    }
    // WGRAD with one split writes dW / db in place (no slab, no reduce pass)
    const bool wdirect = (OP == OP_WGRAD) && a.splits == 1;
    if (do_bias && tid < BM && m0 + tid < M) {
        if (wdirect) a.bias_part[z * a.b_cs + m0 + tid] = bsum;
        else a.bias_part[(int64_t)blockIdx.z * a.M + m0 + tid] = bsum;
    }
    // acc[i][j][r]: row m = (r&3) + 8*(r>>2) + 4*(lane>>5), col n = lane&31.
    const int rbase = 4 * (lane >> 5), col = lane & 31;
    // FWD bias of this lane's output rows, read once (inside the store loop every store
    // forces a re-read: `out` may alias `bias`)
    float bv_r[FM][16];
    if constexpr (OP == OP_FWD) {
        const float* bz = (!partial_out && a.bias) ? a.bias + z * a.b_cs : nullptr;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + rbase;
                bv_r[i][r] = (bz && m < M) ? bz[m] : 0.f;
            }
    }
    const DropKey dkey = drop_key(a.drop, z);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * WN + j * 32 + col;
        if (n >= N) continue;
        if (partial_out) {
            // split-K partial slab part[z][split][m][n] (n over the full-batch extent a.N),
            // or dW itself (row stride N, client stride out_cs)
            float* op = wdirect ? a.out + z * a.out_cs + n
                                : a.out + ((int64_t)blockIdx.z * a.M) * a.N + n;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + rbase;
                    if (m < M) op[(int64_t)m * a.N] = acc[i][j][r];
                }
        } else if constexpr (OP != OP_WGRAD) {
            uint32_t img, p;
            if constexpr (OP == OP_FWD) {
                a.fd_ohw.divmod(n, img, p);
                float* op = a.out + z * a.out_cs + (int64_t)img * a.cout * ohw + p;
                const bool has_bias = a.bias != nullptr;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + rbase;
                        if (m < M) {
                            float v = acc[i][j][r];
                            if (has_bias) v = v + bv_r[i][r];
                            if (a.relu) v = fmaxf(v, 0.f);
                            if (a.drop.mode)
                                v = apply_dropout(a.drop, dkey, z,
                                                  ((int64_t)img * a.cout + m) * ohw + p, v);
                            op[(int64_t)m * ohw] = v;
                        }
                    }
            } else if constexpr (DG2) {
                uint32_t r, c;
                a.fd_ohw.divmod(n, img, p);
                a.fd_ow.divmod(p, r, c);
                float* op = a.out + z * a.out_cs + (int64_t)img * a.cin * hw +
                            (2 * (int)r + py) * a.w + 2 * (int)c + px;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r2 = 0; r2 < 16; ++r2) {
                        const int m = m0 + wm * WM + i * 32 + (r2 & 3) + 8 * (r2 >> 2) + rbase;
                        if (m < M) {
                            float* q = op + (int64_t)m * hw;
                            *q = a.accumulate ? (*q + acc[i][j][r2]) : acc[i][j][r2];
                        }
                    }
            } else {
                a.fd_hw.divmod(n, img, p);
                float* op = a.out + z * a.out_cs + (int64_t)img * a.cin * hw + p;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + rbase;
                        if (m < M) {
                            float* q = op + (int64_t)m * hw;
                            *q = a.accumulate ? (*q + acc[i][j][r]) : acc[i][j][r];
                        }
                    }
            }
        }
    }
}

}  // namespace fh

#include "dconv_kernels.h"

namespace fh {

// Split-K sums of the WGRAD slabs, deterministic (r03).  A thread owns four consecutive
// outputs (one float4 of every split's slab) and one of G contiguous ranges of the splits,
// summed in split order with eight loads in flight; the G range sums are added in range
// order through LDS.  A block covers 256 / G float4s; G grows with the split count (about
// eight splits per thread), so a one-client layer with 128 splits still spreads over
// thousands of threads.  The r02 kernel ran 64 scalar outputs per block (73,728 blocks for
// one 128x8x8 layer of 32 clients: 35 us for 56 MB).
// Blocks past the weight part reduce the conv-bias partials the WGRAD kernel folded in.
template <int G>
__global__ void __launch_bounds__(256)
splitk_sum_kernel(const float* __restrict__ part, float* __restrict__ dw, int64_t dw_cs, int splits,
                  int MN, int wblocks, const float* __restrict__ bpart, float* __restrict__ db,
                  int64_t db_cs, int Mb) {
    constexpr int C = 256 / G;  // float4 columns per block
    __shared__ float4 red[G > 1 ? 256 : 1];
    const int z = blockIdx.y, t = threadIdx.x;
    const bool is_w = (int)blockIdx.x < wblocks;
    const int blk = is_w ? blockIdx.x : blockIdx.x - wblocks;
    const int lim = is_w ? MN : Mb;
    const float* src = is_w ? part + (int64_t)z * splits * MN : bpart + (int64_t)z * splits * Mb;
    const int e0 = (blk * C + t % C) * 4;
    const int piece = t / C;
    const int s0 = (int)((int64_t)splits * piece / G), s1 = (int)((int64_t)splits * (piece + 1) / G);
    const bool vec = (lim & 3) == 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e0 < lim) {
        for (int i0 = s0; i0 < s1; i0 += 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = i0 + j;
                const float* p = src + (int64_t)i * lim + e0;
                if (i >= s1) v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                else if (vec) v[j] = *reinterpret_cast<const float4*>(p);
                else v[j] = make_float4(p[0], e0 + 1 < lim ? p[1] : 0.f, e0 + 2 < lim ? p[2] : 0.f,
                                        e0 + 3 < lim ? p[3] : 0.f);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j < s1) {
                    acc.x += v[j].x;
                    acc.y += v[j].y;
                    acc.z += v[j].z;
                    acc.w += v[j].w;
                }
        }
    }
    if constexpr (G > 1) {
        red[t] = acc;
        __syncthreads();
        if (piece != 0) return;
#pragma unroll
        for (int g = 1; g < G; ++g) {
            const float4 o = red[t + C * g];
            acc.x += o.x;
            acc.y += o.y;
            acc.z += o.z;
            acc.w += o.w;
        }
    }
    if (e0 >= lim) return;
    float* o = is_w ? dw + z * dw_cs + e0 : db + z * db_cs + e0;
    if (vec && ((uintptr_t)o & 15) == 0) {
        *reinterpret_cast<float4*>(o) = acc;
    } else {
        o[0] = acc.x;
        if (e0 + 1 < lim) o[1] = acc.y;
        if (e0 + 2 < lim) o[2] = acc.z;
        if (e0 + 3 < lim) o[3] = acc.w;
    }
}

// the WGRAD reduction launch: dW[z] = sum over splits of part[z][split] (and db from bpart)
static int splitk_sum(const float* part, float* dw, int64_t dw_cs, int splits, int MN,
                      const float* bpart, float* db, int64_t db_cs, int M, int nclients,
                      hipStream_t st) {
    int G = 1;
    while (G < 16 && splits >= 16 * G) G *= 2;  // ~8-15 splits per thread
    const int per = 1024 / G;                   // outputs per block
    const int wblocks = (int)ceil_div(MN, per);
    const int bblocks = db ? (int)ceil_div(M, per) : 0;
    const dim3 grid(wblocks + bblocks, nclients);
#define FH_SKS(GV)                                                                              \
    if (G == GV) {                                                                              \
        FH_LAUNCH(splitk_sum_kernel<GV>, grid, dim3(256), 0, st, part, dw, dw_cs, splits, MN,  \
                  wblocks, bpart, db, db_cs, M);                                                \
        return FH_OK;                                                                           \
    }
    FH_SKS(1)
    FH_SKS(2)
    FH_SKS(4)
    FH_SKS(8)
    FH_SKS(16)
#undef FH_SKS
    return FH_E_UNSUPPORTED;
}

// DGRAD split-K epilogue with BatchNorm backward statistics (DConvArgs::bnx and friends)
struct BnBwdEpi {
    const float* x;  // nullptr: off
    int64_t x_cs;
    const float* scale;
    const float* shift;
    int64_t s_cs;
    const float* mean;
    const uint8_t* pidx;  // non-null: routed through a 2x2 max-pool (+ dropout)
    const uint8_t* pmask;
    int64_t pi_cs, pm_cs;
    float pscale;
    int pw;  // pooled map width (the epilogue's map), x is 2pw wide
};

// FWD split-K epilogue with the 2x2 max-pool after the ReLU (fh_conv2d_fwd_relu_pool on a
// split launch): planes of 256 pixels (one image per workgroup), the pool of the top-left
// hw x hw map of each -> y [img][M][hw/2][hw/2] + argmax (maxpool2_fwd_kernel's rule); the
// un-pooled output is not stored
struct PoolEpi {
    float* y;  // nullptr: off
    uint8_t* idx;
    int64_t y_cs, i_cs;
    int hw, w;  // pooled map size, plane width
};

// FWD/DGRAD split-K epilogue: out[z][img][m][p] (=|+=) sum_s part[z][s][m][n] (+bias, relu).
// bn_part (nullable): one fp64 pair per (client, channel, 256-pixel tile) as the unsplit
// dconv epilogue writes it (dconv_kernels.h DConvArgs::bn_part): FWD the BatchNorm
// statistics (sum, sum of squares) of the stored values; DGRAD with bb.x the BN backward
// statistics (sum g, sum (x - mean) g) of the ReLU-masked gradient g it stores.
__global__ void __launch_bounds__(256)
splitk_epilogue_kernel(const float* __restrict__ part, int splits, int M, int Nfull,
                       float* __restrict__ out, int64_t out_cs, const float* __restrict__ bias,
                       int64_t b_cs, int relu, int accumulate, const int32_t* __restrict__ counts,
                       int batch, int sp, double* __restrict__ bn_part, int bn_tiles,
                       DropArgs drop, BnBwdEpi bb, PoolEpi pe) {
    const int z = blockIdx.z, m = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int n = blockIdx.x * 256 + threadIdx.x;
    const bool valid = n < cnt * sp;
    if (!valid && bn_part == nullptr) return;  // with pe.y (sp = 256): block-uniform
    float s = 0.f, d0f = 0.f, d1f = 0.f;
    if (valid) {
        const float* p = part + ((int64_t)z * splits * M + m) * Nfull + n;
        const int64_t ss = (int64_t)M * Nfull;
        for (int i0 = 0; i0 < splits; i0 += 8) {  // 8 loads in flight, summed in split order
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = i0 + j < splits ? p[(i0 + j) * ss] : 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j < splits) s += v[j];
        }
        if (bias) s = s + bias[z * b_cs + m];
        if (relu) s = fmaxf(s, 0.f);
        const int img = n / sp, pix = n - img * sp;
        if (drop.mode) s = apply_dropout(drop, drop_key(drop, z), z, ((int64_t)img * M + m) * sp + pix, s);
        float* o = out + z * out_cs + ((int64_t)img * M + m) * sp + pix;
        if (accumulate) s = *o + s;
        if (bb.x) {  // ReLU mask of the BN in front; (x - mean) * g for its statistics
            const int64_t e = ((int64_t)img * M + m) * sp + pix;
            float xv, gu = s;
            if (bb.pidx) {
                const int code = bb.pidx[z * bb.pi_cs + e];
                if (bb.pmask) gu = bb.pmask[z * bb.pm_cs + e] ? s * bb.pscale : 0.f;
                const int py = pix / bb.pw, px = pix - py * bb.pw;
                xv = bb.x[z * bb.x_cs + ((int64_t)img * M + m) * 4 * sp +
                          (2 * py + (code >> 1)) * (2 * bb.pw) + 2 * px + (code & 1)];
            } else {
                xv = bb.x[z * bb.x_cs + e];
            }
            const float g =
                (xv * bb.scale[z * bb.s_cs + m] + bb.shift[z * bb.s_cs + m] > 0.f) ? gu : 0.f;
            d0f = g;
            d1f = (xv - bb.mean[z * M + m]) * g;
            if (!bb.pidx) s = g;
        }
        if (!pe.y) *o = s;
    }
    if (pe.y) {  // block-uniform; the workgroup is one image's channel-m plane
        __shared__ float pl[256];
        pl[threadIdx.x] = s;
        __syncthreads();
        const int ph = pe.hw >> 1, per = ph * ph;
        if ((int)threadIdx.x < per) {
            const int oy = threadIdx.x / ph, ox = threadIdx.x - oy * ph;
            const float* r = pl + (2 * oy) * pe.w + 2 * ox;
            const float v0 = r[0], v1 = r[1], v2 = r[pe.w], v3 = r[pe.w + 1];
            float mx = v0;
            int am = 0;
            if (v1 > mx) { mx = v1; am = 1; }
            if (v2 > mx) { mx = v2; am = 2; }
            if (v3 > mx) { mx = v3; am = 3; }
            const int img = n / sp;
            const int64_t o = ((int64_t)img * M + m) * per + threadIdx.x;
            pe.y[z * pe.y_cs + o] = mx;
            pe.idx[z * pe.i_cs + o] = (uint8_t)am;
        }
    }
    if (bn_part != nullptr) {  // block-uniform
        __shared__ double red[2][4];
        double d0 = !valid ? 0.0 : bb.x ? (double)d0f : (double)s;
        double d1 = bb.x ? (double)d1f : d0 * d0;
        d0 = wave_sum(d0);
        d1 = wave_sum(d1);
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (lane == 0) {
            red[0][wid] = d0;
            red[1][wid] = d1;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* q = bn_part + (((int64_t)z * M + m) * bn_tiles + blockIdx.x) * 2;
            q[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
            q[1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
        }
    }
}

// OP_DGRAD_S2 split-K epilogue: slab part[(client*4 + phase)][split][m][n over the phase
// grid] summed in split order into dX[client][img][m][2oy'+py][2ox'+px] (=|+=).
__global__ void __launch_bounds__(256)
splitk_epilogue_s2_kernel(const float* __restrict__ part, int splits, int M, int Nfull,
                          float* __restrict__ out, int64_t out_cs, int accumulate,
                          const int32_t* __restrict__ counts, int batch, int oh, int ow, int w) {
    const int zz = blockIdx.z, z = zz >> 2, py = (zz >> 1) & 1, px = zz & 1, m = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int ohw = oh * ow;
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= cnt * ohw) return;
    const float* p = part + ((int64_t)zz * splits * M + m) * Nfull + n;
    const int64_t ss = (int64_t)M * Nfull;
    float s = 0.f;
    for (int i0 = 0; i0 < splits; i0 += 8) {  // 8 loads in flight, summed in split order
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = i0 + j < splits ? p[(i0 + j) * ss] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (i0 + j < splits) s += v[j];
    }
    const int img = n / ohw, q = n - img * ohw, r = q / ow, c = q - r * ow;
    float* o = out + z * out_cs + ((int64_t)img * M + m) * (4 * ohw) + (2 * r + py) * w + 2 * c + px;
    *o = accumulate ? (*o + s) : s;
}

// ---------------------------------------------------------------------------
// Single-input-channel 3x3 / stride 1 / pad 1 convolution (SimpleCNN conv1 on 28x28 MNIST
// maps, models_pytorch.py:66-70) — K = 9, so an implicit GEMM spends its time on operand
// gathers and a 16-deep k tile that is mostly zeros.  FWD: one thread per output pixel, its
// 9 input taps in registers, the COUT x 9 weights + bias in LDS; y stores coalesced per
// channel (the layer is bound by writing y).  WGRAD: a block = 8 output channels x a chunk of
// the client's pixels, each thread 8 x 9 tap products + 8 bias terms in registers, a fixed-
// order wave / block reduction into a per-chunk slab reduced by splitk_sum_kernel.
constexpr int kC1Chunk = 2048;  // WGRAD pixels per block (8 per thread, loads 4 pixels ahead)

template <int COUT>
__global__ void __launch_bounds__(256)
conv_c1_fwd_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ w,
                   int64_t w_cs, const float* __restrict__ bias, int64_t b_cs,
                   float* __restrict__ y, int64_t y_cs, const int32_t* __restrict__ counts,
                   int batch, int H, int W, int relu) {
    __shared__ float ws[COUT * 9], bs[COUT];
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    for (int i = threadIdx.x; i < COUT * 9; i += 256) ws[i] = w[z * w_cs + i];
    for (int i = threadIdx.x; i < COUT; i += 256) bs[i] = bias ? bias[z * b_cs + i] : 0.f;
    __syncthreads();
    const int HW = H * W;
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= cnt * HW) return;
    const int img = n / HW, p = n - img * HW, r = p / W, c = p - r * W;
    const float* xi = x + z * x_cs + (int64_t)img * HW;
    float t[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int yy = r + kh - 1, xx = c + kw - 1;
            t[kh * 3 + kw] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                                 ? xi[yy * W + xx] : 0.f;
        }
    float* yo = y + z * y_cs + (int64_t)img * COUT * HW + p;
#pragma unroll 4
    for (int co = 0; co < COUT; ++co) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) v = fmaf(ws[co * 9 + k], t[k], v);
        v = v + bs[co];
        if (relu) v = fmaxf(v, 0.f);
        yo[(int64_t)co * HW] = v;
    }
}

// conv_c1_fwd_kernel (+ bias, ReLU) fused with the 2x2 max-pool after it (SimpleCNN conv1 ->
// ReLU -> pool1, models_pytorch.py:80-82): one thread per POOLED pixel computes its 2x2 window
// of conv outputs per channel with conv_c1_fwd_kernel's operations and pools them as
// maxpool2_fwd_kernel does (strict >, window order) -> y (pooled planes yh x yw, the map in the
// top-left corner) and the uint8 argmax idx; the full-resolution ReLU output is never written
// (the backward's ReLU mask at the argmax is y > 0: conv_c1_wgrad_kernel<true>).
// U8Src (non-null data): the input is read from the raw uint8 images instead of x — the
// step's batch gather (fh_gather_u8: x = (u / 255 - mean) / std, no crop / flip, one channel)
// folded into this launch: x is still written (each thread its own 2x2 window's pixels, for the
// weight gradient's and the evaluation's reads) and so are the labels (r04, one launch less
// per SimpleCNN step)
struct U8Src {
    const uint8_t* data;    // [N][H][W]
    const int64_t* labels;  // [N]
    const int64_t* gidx;    // [z][batch] sample of each batch slot
    int64_t g_cs;
    int64_t* ylab;          // [z][batch] labels out
    int64_t yl_cs;
    float mean, stdv;
    float* xo;              // x written (the kernel's x parameter is read-only: not read here)
    int64_t xo_cs;
};

// r05: a workgroup takes one group of CG channels (blockIdx.y) of one client (blockIdx.z), so
// the weights and bias are workgroup-uniform: scalar loads, the FMAs take them as SGPR operands
// (r02-r04 staged all COUT x 9 in LDS and read them back per channel).  CG = 8 on narrow
// launches (a one-client launch runs COUT / 8 times the workgroups: K2's one-client conv1
// 14.9 -> 11.4 us), CG = COUT from kC1PoolWide clients on (the patch is loaded once per pixel:
// the 8-channel groups re-read it and were 3 % slower at 9-32 clients).  Each thread computes
// one pooled pixel's window with the same fmaf order per channel; with U8Src only the first
// channel group writes x and the labels (every group reads the bytes).
constexpr int kC1PoolWide = 8;
template <int COUT, int CG>
__global__ void __launch_bounds__(256)
conv_c1_pool_fwd_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ w,
                        int64_t w_cs, const float* __restrict__ bias, int64_t b_cs,
                        float* __restrict__ y, int64_t y_cs, uint8_t* __restrict__ idx,
                        int64_t i_cs, const int32_t* __restrict__ counts, int batch, int H,
                        int W, int yh, int yw, const U8Src src) {
    const int z = blockIdx.z, cg = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int OH = H / 2, OW = W / 2, OHW = OH * OW;
    const int n = blockIdx.x * 256 + threadIdx.x;
    if (n >= cnt * OHW) return;
    const int img = n / OHW, q = n - img * OHW, oh = q / OW, ow = q - oh * OW;
    const float* xi = x + z * x_cs + (int64_t)img * H * W;
    float t[4][4];  // input rows 2oh-1 .. 2oh+2, columns 2ow-1 .. 2ow+2 (zero padding)
    if (src.data) {  // the gather folded in: gather_u8_kernel's operations on the raw bytes
        const int64_t s = src.gidx[z * src.g_cs + img];
        const uint8_t* si = src.data + s * H * W;
        float* xo = src.xo + z * src.xo_cs + (int64_t)img * H * W;
        const bool wr = cg == 0;
        // every byte (and the label) loaded before the first x store (r05: xo may alias the
        // bytes for the compiler, so each later load waited for the stores before it — a
        // dependent global round trip per window row)
        uint32_t b[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int yy = 2 * oh + i - 1, xx = 2 * ow + j - 1;
                b[i][j] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                              ? (uint32_t)si[yy * W + xx] : 0x100u;  // 0x100: padding
            }
        const int64_t lab = wr && q == 0 ? src.labels[s] : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = 0.f;
                if (b[i][j] < 0x100u) {
                    const float u = __fdiv_rn((float)b[i][j], 255.f);
                    v = __fdiv_rn(u - src.mean, src.stdv);
                }
                t[i][j] = v;
            }
        if (wr) {
#pragma unroll
            for (int i = 1; i <= 2; ++i)
#pragma unroll
                for (int j = 1; j <= 2; ++j) {  // own window: always inside the image
                    const int yy = 2 * oh + i - 1, xx = 2 * ow + j - 1;
                    xo[yy * W + xx] = t[i][j];
                }
            if (q == 0) src.ylab[z * src.yl_cs + img] = lab;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int yy = 2 * oh + i - 1, xx = 2 * ow + j - 1;
                t[i][j] = ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                              ? xi[yy * W + xx]
                              : 0.f;
            }
    }
    const int c0 = cg * CG;
    const float* wz = w + z * w_cs + c0 * 9;  // workgroup-uniform: scalar loads
    const float* bz = bias ? bias + z * b_cs + c0 : nullptr;
    float* yo = y + z * y_cs + ((int64_t)img * COUT + c0) * yh * yw + oh * yw + ow;
    uint8_t* io = idx + z * i_cs + ((int64_t)img * COUT + c0) * OHW + q;
#pragma unroll(CG == COUT ? 2 : CG)
    for (int c = 0; c < CG; ++c) {
        float v[4];
        const float bc = bz ? bz[c] : 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s) {  // window slot s = (dy, dx) = (s >> 1, s & 1)
            float a = 0.f;
#pragma unroll
            for (int k = 0; k < 9; ++k)
                a = fmaf(wz[c * 9 + k], t[(s >> 1) + k / 3][(s & 1) + k % 3], a);
            a = a + bc;
            v[s] = fmaxf(a, 0.f);
        }
        float m = v[0];
        int am = 0;
        if (v[1] > m) { m = v[1]; am = 1; }
        if (v[2] > m) { m = v[2]; am = 2; }
        if (v[3] > m) { m = v[3]; am = 3; }
        yo[(int64_t)c * yh * yw] = m;
        io[(int64_t)c * OHW] = (uint8_t)am;
    }
}

// part[z][chunk][co*9 + k], bpart[z][chunk][co]  (dwgrad_ws_bytes layout, splits = chunks).
// POOLED: dy is not materialised — the gradient of pixel (r, c) is the pooled gradient
// gp[r/2][c/2] (planes gh x gw) if (r, c) is its window's argmax and the pooled ReLU output
// yp there is > 0, else 0: maxpool2_bwd_kernel's routing and ReLU mask (xin at the argmax is
// the pooled value), so the products are the same as on its output.
template <bool POOLED>
__global__ void __launch_bounds__(256)
conv_c1_wgrad_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ dy,
                     int64_t dy_cs, float* __restrict__ part, float* __restrict__ bpart,
                     const int32_t* __restrict__ counts, int batch, int H, int W, int cout,
                     int nchunks, const uint8_t* __restrict__ pidx, int64_t pi_cs,
                     const float* __restrict__ yp, int64_t yp_cs, int gh, int gw) {
    __shared__ float red[4][8 * 10];
    const int chunk = blockIdx.x, cg = blockIdx.y, z = blockIdx.z;
    const int cnt = counts ? counts[z] : batch;
    const int HW = H * W;
    const int n0 = chunk * kC1Chunk, n1 = min(cnt * HW, n0 + kC1Chunk);
    float acc[8][10];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) acc[j][k] = 0.f;
    const float* xz = x + z * x_cs;
    const float* dz = dy + z * dy_cs + (int64_t)cg * 8 * HW;
    // four pixels per pass, all their loads issued before the FMAs (the loop is bound by load
    // latency, not by the 80 FMAs a pixel costs); pixels past the chunk contribute zeros
    constexpr int U = 4;
    for (int nb = n0 + threadIdx.x; nb < n1; nb += U * 256) {
        float t[U][9], g[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int n = nb + u * 256;
            const bool ok = n < n1;
            const int nn = ok ? n : n0;
            const int img = nn / HW, p = nn - img * HW, r = p / W, c = p - r * W;
            const float* xi = xz + (int64_t)img * HW;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh)
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const int yy = r + kh - 1, xx = c + kw - 1;
                    t[u][kh * 3 + kw] =
                        (ok && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W)
                            ? xi[yy * W + xx] : 0.f;
                }
            if constexpr (POOLED) {
                const int OH = H / 2, OW = W / 2;
                const int oh = r >> 1, ow = c >> 1, code = (r & 1) * 2 + (c & 1);
                const int64_t pl = (int64_t)img * cout + cg * 8;
                const uint8_t* ii = pidx + z * pi_cs + pl * OH * OW + oh * OW + ow;
                const int64_t gq = pl * gh * gw + oh * gw + ow;
                const float* gi = dy + z * dy_cs + gq;
                const float* yi = yp + z * yp_cs + gq;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool hit = ok && ii[(int64_t)j * OH * OW] == code &&
                                     yi[(int64_t)j * gh * gw] > 0.f;
                    g[u][j] = hit ? gi[(int64_t)j * gh * gw] : 0.f;
                }
            } else {
                const float* di = dz + (int64_t)img * cout * HW + p;
#pragma unroll
                for (int j = 0; j < 8; ++j) g[u][j] = ok ? di[(int64_t)j * HW] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int k = 0; k < 9; ++k) acc[j][k] = fmaf(g[u][j], t[u][k], acc[j][k]);
                acc[j][9] += g[u][j];
            }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const float v = wave_sum(acc[j][k]);
            if (lane == 0) red[wid][j * 10 + k] = v;
        }
    __syncthreads();
    if (threadIdx.x < 80) {
        const int j = threadIdx.x / 10, k = threadIdx.x % 10;
        const float v = (red[0][threadIdx.x] + red[1][threadIdx.x]) +
                        (red[2][threadIdx.x] + red[3][threadIdx.x]);
        const int co = cg * 8 + j;
        const int64_t slab = (int64_t)z * nchunks + chunk;
        if (k < 9) part[slab * cout * 9 + co * 9 + k] = v;
        else if (bpart) bpart[slab * cout + co] = v;
    }
}

// SimpleCNN conv1 WGRAD on the matrix cores (r03).  dW[co][tap] = sum_px dY[co][px] T[px][tap]
// is a GEMM with a long pixel reduction: M = COUT, N = 16 taps (the 9 shifts, tap 9 = 1.0 gives
// the bias gradient, taps 10-15 zero), K = pixels, one v_mfma_f32_16x16x4_f32 per 16 output
// channels and 4 pixels.  A workgroup takes a run of 4-row stages of one client (dY [COUT][4
// rows] and the 6 input rows with a zero halo staged in LDS, pitches = 2 (mod 4)); wave w
// multiplies stage row w, so per stage a wave issues W/4 x COUT/16 MFMAs from one patch read
// (per-lane tap offset) and COUT/16 dY reads per 4 pixels.  The four waves' sums are added
// in wave order at the end; splits of the stage run land in the same slab as
// conv_c1_wgrad_kernel (splitk_sum).  The VALU kernel it replaces (80 fmaf per pixel per
// 8 channels, runtime divisions per pixel) moved 1.3 TB/s at 32 clients (79.7 us).
// H % 4 == 0, W % 4 == 0, W <= 32.
// POOLED: dY is not materialised — it is routed from the pooled gradient as
// maxpool2_bwd_ymask does (conv_c1_wgrad_kernel<true> above): pixel (y, x) takes dpool[y/2][x/2]
// (planes gh x gw) when it is its window's argmax (idx, dense) and the pooled ReLU output yp
// there is > 0, else 0 — per staged quad two pooled values, two argmax bytes, two yp values.
// The same fp32 values reach the same MFMA chain, so the result equals the unfused pair
// (maxpool2_bwd_ymask + this kernel on its output) bit for bit.
constexpr int kNormSrcMax = 4;
struct NormSrcs {
    fh_linear_norm_src lin[kNormSrcMax];
    int nlin;
    const float* sw[kNormSrcMax];  // slab weights [z][i][per_w]
    const float* sb[kNormSrcMax];  // slab bias [z][i][per_b] (nullable)
    int per_w[kNormSrcMax], per_b[kNormSrcMax];
    int nslab;
};

// Image i of client z: its squared gradient norm over every layer — linear layers by the rank-1
// identity ||dy_i||^2 (||x_i||^2 + bias), conv layers as the sum of squares of the image's slab
// rows — in fp64, then its clip coefficient (clip_coef_kernel's arithmetic).  The body of
// dpsgd_norm_clip_kernel (one workgroup per (image, client)) and, r05, the tail of the per-image
// conv1 slab launch (conv_c1_wgrad_mfma_kernel<..., NORM>), which runs the same code on the same
// grid after its own slab row is written: the same sums, one launch less per DP-SGD step.
__device__ __forceinline__ void dpsgd_norm_clip_body(const NormSrcs& src, int cnt, int batch,
                                                     double max_norm, double* __restrict__ sqnorm,
                                                     float* __restrict__ coef, int i, int z,
                                                     double* red) {
    const int64_t row = (int64_t)z * batch + i;
    if (i >= cnt) {  // block-uniform
        if (threadIdx.x == 0) {
            coef[row] = 0.f;
            if (sqnorm) sqnorm[row] = 0.0;
        }
        return;
    }
    double total = 0.0;
    for (int l = 0; l < src.nlin; ++l) {
        const fh_linear_norm_src& L = src.lin[l];
        const float* xr = L.x + z * L.x_cs + (int64_t)i * L.in_f;
        const float* dr = L.dy + z * L.dy_cs + (int64_t)i * L.out_f;
        double sx = 0.0, sd = 0.0;
        // unrolled loops keep each thread's order (the same sums) with several loads in flight
#pragma unroll 4
        for (int k = threadIdx.x; k < L.in_f; k += 256) sx += (double)xr[k] * (double)xr[k];
#pragma unroll 4
        for (int k = threadIdx.x; k < L.out_f; k += 256) sd += (double)dr[k] * (double)dr[k];
        sx = block_sum_256(sx, red);
        sd = block_sum_256(sd, red);
        total += sd * (sx + (L.with_bias ? 1.0 : 0.0));
    }
    for (int l = 0; l < src.nslab; ++l) {
        const float4* w4 = reinterpret_cast<const float4*>(src.sw[l] + row * src.per_w[l]);
        double sq = 0.0;
#pragma unroll 4
        for (int q = threadIdx.x; q < src.per_w[l] / 4; q += 256) {
            const float4 v = w4[q];
            sq += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        }
        if (src.sb[l])
            for (int q = threadIdx.x; q < src.per_b[l]; q += 256) {
                const double v = src.sb[l][row * src.per_b[l] + q];
                sq += v * v;
            }
        total += block_sum_256(sq, red);
    }
    if (threadIdx.x == 0) {
        if (sqnorm) sqnorm[row] = total;
        // ||g_i|| = B * ||g_i / B||  (the stored gradients are of the batch-mean loss)
        const double norm = (double)cnt * sqrt(total);
        coef[row] = norm > max_norm ? (float)(max_norm / norm) : 1.0f;
    }
}

__global__ void __launch_bounds__(256)
dpsgd_norm_clip_kernel(const NormSrcs src, const int32_t* __restrict__ counts, int batch,
                       double max_norm, double* __restrict__ sqnorm, float* __restrict__ coef) {
    __shared__ double red[4];
    const int i = blockIdx.x, z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    dpsgd_norm_clip_body(src, cnt, batch, max_norm, sqnorm, coef, i, z, red);
}

// a split DGRAD's partial slab read in place of its reduced output (fh_conv_defer_dgrad, r05):
// element (img, c, y, x) of the dX planes (256-pixel planes) is
// sum_s p[((z * splits + s) * M + c) * Nfull + img * 256 + y * 16 + x], summed as
// splitk_epilogue_kernel sums it (0 + p0 + p1 + ... in split order): the same bits
struct DgradParts {
    const float* p;  // nullptr: off
    int splits, M;
    int64_t Nfull;
};
constexpr int kDgradPartsMax = 4;  // kDconvMaxSplits

// the norm / clip tail of the per-image conv1 slab launch (NORM instances)
struct NormTail {
    NormSrcs src;
    double max_norm;
    double* sqnorm;
    float* coef;
};

template <int COUT, bool POOLED, int NS = 2, bool NORM = false, int NP = 0>
__global__ void __launch_bounds__(256)
conv_c1_wgrad_mfma_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ dy,
                          int64_t dy_cs, float* part, float* bpart,
                          const int32_t* __restrict__ counts, int batch, int H, int W,
                          int nsplits, int sps, const uint8_t* __restrict__ pidx, int64_t pi_cs,
                          const float* __restrict__ yp, int64_t yp_cs, int gh, int gw,
                          const NormTail tail, const DgradParts dp) {
    // part / bpart carry no __restrict__: the NORM instance reads its own slab row back through
    // tail.src after the workgroup barrier (they are only written in the epilogue, so the main
    // loop's scheduling does not depend on it)
    constexpr int NQ = COUT / 16;     // 16-channel groups
    constexpr int MAXW = 32;
    constexpr int DP = 4 * MAXW + 2;  // dY pitch per channel (4 rows), = 2 (mod 4)
    constexpr int PW = MAXW + 4;      // patch row pitch: image column c at 2 + c
    constexpr int NDQ = COUT * MAXW / 256;  // dY float4s per thread (upper bound)
    // r05: NS 4-row stages per LDS round (one load round trip and two barriers per NS stages:
    // the one-stage rounds waited a full memory latency for 14 MFMAs each); the pixel order of
    // the MFMA chain is unchanged, so the sums are the same bits.  NS = 2 (40 KB of LDS, four
    // workgroups per CU); NS = 4 for the per-image DP-SGD slabs on narrow grids (75 KB: seven
    // stages = one image in two rounds)
    __shared__ float Ds[NS][COUT * DP];
    __shared__ float Ps[NS][6 * PW];
    __shared__ float red[4][COUT * 10];
    const int split = blockIdx.x, z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int HW = H * W, Q = W / 4;
    const int nst = cnt * (H / 4);
    const int sbeg = split * sps, send = min(nst, sbeg + sps);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const float* xz = x + z * x_cs;
    const float* dyz = dy + z * dy_cs;
    if (tid < 6 * NS) {  // zero halo columns -1 and W (never overwritten)
        Ps[tid / 6][(tid % 6) * PW + 1] = 0.f;
        Ps[tid / 6][(tid % 6) * PW + W + 2] = 0.f;
    }
    const int nd4 = COUT * 4 * Q;
    float4 rd[NS][NDQ], rx[NS];
    float2 pq[NS][POOLED ? NDQ : 1][NP > 0 ? NP : 1];  // NP: deferred DGRAD partials (dp.p)
    float2 pg[NS][POOLED ? NDQ : 1], py[NS][POOLED ? NDQ : 1];  // POOLED: raw loads, routed
    int pc[NS][POOLED ? NDQ : 1];                    // in store(); argmax bytes | code row << 16
    auto load = [&](int st0) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const int st = st0 + u;
            const bool live = st < send;
            const int img = (4 * st) / H, y0 = (4 * st) % H;
#pragma unroll
            for (int i = 0; i < NDQ; ++i) {
                const int q = tid + 256 * i;
                const int co = q / (4 * Q), rem = q % (4 * Q), rr = rem / Q, qq = rem % Q;
                const bool ok = live && q < nd4;
                if constexpr (POOLED) {
                    const int yy = y0 + rr, OHW = (H / 2) * (W / 2);
                    const int64_t pl = (int64_t)img * COUT + co;
                    const int64_t go = pl * gh * gw + (yy >> 1) * gw + 2 * qq;
                    const int64_t io = pl * OHW + (yy >> 1) * (W / 2) + 2 * qq;
                    if (NP > 0 && dp.p) {  // the partials of the deferred DGRAD reduction
                        const int64_t po = ((int64_t)z * dp.splits * dp.M + co) * dp.Nfull +
                                           (int64_t)img * (gh * gw) + (yy >> 1) * gw + 2 * qq;
                        const int64_t ss = (int64_t)dp.M * dp.Nfull;
#pragma unroll
                        for (int sp = 0; sp < NP; ++sp) {
                            const int64_t o = ok && sp < dp.splits ? po + sp * ss : 0;
                            pq[u][i][sp] = make_float2(dp.p[o], dp.p[o + 1]);
                        }
                    }
                    pg[u][i] = make_float2(0.f, 0.f);
                    if (!(NP > 0 && dp.p) && ok) pg[u][i] = make_float2(dyz[go], dyz[go + 1]);
                    py[u][i] = ok ? make_float2(yp[z * yp_cs + go], yp[z * yp_cs + go + 1])
                                  : make_float2(0.f, 0.f);
                    pc[u][i] = ok ? (pidx[z * pi_cs + io] | (pidx[z * pi_cs + io + 1] << 8) |
                                     ((yy & 1) << 17) | (1 << 24))  // bit 24: a live quad
                                  : 0;
                } else {
                    rd[u][i] = ok ? *reinterpret_cast<const float4*>(
                                        dyz + ((int64_t)(img * COUT + co) * HW + (y0 + rr) * W +
                                               4 * qq))
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            rx[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (tid < 6 * Q) {
                const int pr = tid / Q, qq = tid % Q, y = y0 + pr - 1;
                if (live && (unsigned)y < (unsigned)H)
                    rx[u] = *reinterpret_cast<const float4*>(xz + (int64_t)img * HW + y * W + 4 * qq);
            }
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
#pragma unroll
            for (int i = 0; i < NDQ; ++i) {
                const int q = tid + 256 * i;
                if constexpr (POOLED) {  // maxpool2_bwd_kernel's routing: (code == a) ? g : 0
                    if (NP > 0 && dp.p) {  // splitk_epilogue_kernel's sum: 0 + p0 + p1 + ...
                        float2 g = make_float2(0.f, 0.f);
#pragma unroll
                        for (int sp = 0; sp < NP; ++sp)
                            if (sp < dp.splits) {
                                g.x += pq[u][i][sp].x;
                                g.y += pq[u][i][sp].y;
                            }
                        pg[u][i] = (pc[u][i] >> 24) & 1 ? g : make_float2(0.f, 0.f);
                    }
                    const int c = pc[u][i];
                    const int r = (c >> 16) & 0xff, i0 = c & 0xff, i1 = (c >> 8) & 0xff;
                    const float g0 = py[u][i].x > 0.f ? pg[u][i].x : 0.f;
                    const float g1 = py[u][i].y > 0.f ? pg[u][i].y : 0.f;
                    rd[u][i] = make_float4(i0 == r ? g0 : 0.f, i0 == (r | 1) ? g0 : 0.f,
                                           i1 == r ? g1 : 0.f, i1 == (r | 1) ? g1 : 0.f);
                }
                if (q < nd4) {
                    const int co = q / (4 * Q), rem = q % (4 * Q), rr = rem / Q, qq = rem % Q;
                    float2* d = reinterpret_cast<float2*>(&Ds[u][co * DP + rr * W + 4 * qq]);
                    d[0] = make_float2(rd[u][i].x, rd[u][i].y);
                    d[1] = make_float2(rd[u][i].z, rd[u][i].w);
                }
            }
            if (tid < 6 * Q) {
                const int pr = tid / Q, qq = tid % Q;
                float2* d = reinterpret_cast<float2*>(&Ps[u][pr * PW + 2 + 4 * qq]);
                d[0] = make_float2(rx[u].x, rx[u].y);
                d[1] = make_float2(rx[u].z, rx[u].w);
            }
        }
    };
    // lane roles: m / n = lane & 15 (channel of the A operand / tap of the B operand),
    // k = lane >> 4 (pixel of the 4-pixel group)
    const int mn = lane & 15, kk = lane >> 4;
    const int toff = mn < 9 ? (mn / 3) * PW + mn % 3 + 1 : 0;
    const float tconst = mn == 9 ? 1.f : 0.f;
    f32x4 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (sbeg < send) {
        load(sbeg);
        store();
        __syncthreads();
        for (int st = sbeg; st < send; st += NS) {
            const bool more = st + NS < send;
            if (more) load(st + NS);
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                if (st + u < send) {  // block-uniform
                    const float* Pr = &Ps[u][wid * PW + kk + toff];
                    const float* Dr = &Ds[u][mn * DP + wid * W + kk];
                    for (int g = 0; g < Q; ++g) {
                        const float b = mn < 9 ? Pr[4 * g] : tconst;
#pragma unroll
                        for (int q = 0; q < NQ; ++q)
                            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(Dr[q * 16 * DP + 4 * g], b,
                                                                          acc[q], 0, 0, 0);
                    }
                }
            }
            if (more) {
                __syncthreads();
                store();
                __syncthreads();
            }
        }
    }
    // D[co][tap]: lane holds taps mn, channels q*16 + 4*kk + r
    if (mn < 10) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wid][(q * 16 + 4 * kk + r) * 10 + mn] = acc[q][r];
    }
    __syncthreads();
    const int64_t slab = (int64_t)z * nsplits + split;
    for (int e = tid; e < COUT * 10; e += 256) {
        const float v = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
        const int co = e / 10, k = e % 10;
        if (k < 9) part[slab * COUT * 9 + co * 9 + k] = v;
        else if (bpart) bpart[slab * COUT + co] = v;
    }
    if constexpr (NORM) {
        // one split = one image (the per-image launch): its slab row is written above; after
        // a workgroup-scope release / barrier every thread reads it back with the other layers'
        // sources (written by earlier launches) for the image's norm and clip coefficient
        __shared__ double nred[4];
        __threadfence_block();
        __syncthreads();
        dpsgd_norm_clip_body(tail.src, cnt, nsplits, tail.max_norm, tail.sqnorm, tail.coef,
                             split, z, nred);
    }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
struct Tile {
    int bm, bn, bk, wavesm;
};

template <int OP, int KH, int KW, int S>
static int launch_tile(const Tile& t, dim3 grid, const ConvArgs& a, hipStream_t st) {
#define FH_IG(BM, BN, BK, WMV)                                                               \
    if (t.bm == BM && t.bn == BN && t.bk == BK && t.wavesm == WMV) {                         \
        FH_LAUNCH((igemm_kernel<OP, KH, KW, S, BM, BN, BK, WMV>), grid, dim3(256), 0, \
                           st, a);                                                           \
        return FH_OK;                                                                        \
    }
    if constexpr (OP == OP_WGRAD) {
        FH_IG(32, 128, 32, 1)
        FH_IG(64, 128, 32, 2)
        FH_IG(128, 128, 32, 2)
    } else {
        FH_IG(32, 256, 16, 1)
        FH_IG(64, 256, 16, 1)
        FH_IG(128, 128, 16, 2)
        FH_IG(128, 32, 16, 4)
    }
#undef FH_IG
    set_error("igemm: no tile instantiation (%d,%d,%d,%d)", t.bm, t.bn, t.bk, t.wavesm);
    return FH_E_UNSUPPORTED;
}

template <int OP>
static int launch_shape(int kh, int kw, int s, const Tile& t, dim3 grid, const ConvArgs& a,
                        hipStream_t st) {
    if constexpr (OP == OP_DGRAD_S2) {
        if (kh == 3 && kw == 3 && s == 2) return launch_tile<OP, 3, 3, 2>(t, grid, a, st);
        if (kh == 1 && kw == 1 && s == 2) return launch_tile<OP, 1, 1, 2>(t, grid, a, st);
        set_error("conv dgrad s2: unsupported kernel %dx%d stride %d", kh, kw, s);
        return FH_E_UNSUPPORTED;
    }
    if (kh == 3 && kw == 3 && s == 1) return launch_tile<OP, 3, 3, 1>(t, grid, a, st);
    if (kh == 3 && kw == 3 && s == 2) return launch_tile<OP, 3, 3, 2>(t, grid, a, st);
    if (kh == 1 && kw == 1 && s == 1) return launch_tile<OP, 1, 1, 1>(t, grid, a, st);
    if (kh == 1 && kw == 1 && s == 2) return launch_tile<OP, 1, 1, 2>(t, grid, a, st);
    set_error("conv: unsupported kernel %dx%d stride %d", kh, kw, s);
    return FH_E_UNSUPPORTED;
}

static Tile pick_mn_tile(int M, int Nmax) {
    if (Nmax <= 32) return {128, 32, 16, 4};
    if (M <= 32) return {32, 256, 16, 1};
    if (M <= 64) return {64, 256, 16, 1};
    return {128, 128, 16, 2};
}

static Tile pick_wgrad_tile(int M) {
    if (M <= 32) return {32, 128, 32, 1};
    if (M <= 64) return {64, 128, 32, 2};
    return {128, 128, 32, 2};
}

// Fill fraction (thread-local, fh_set_fill_fraction): the share of the chip one launch
// should aim to fill when it splits K.  1 = the whole chip (a lone packed lane); a lane
// that runs concurrently with others (fedhip/lanes.py) asks for less, trading split-K
// partial slabs and their epilogue launches for longer, fuller workgroups.
static thread_local float g_fill = 1.0f;
static int64_t fill(int64_t workgroups) {
    return std::max<int64_t>(1, (int64_t)((double)workgroups * g_fill));
}

// Split K so that (tiles x splits) fills the chip, each split keeping >= min_chunks K-steps.
static void choose_split(int64_t tiles, int K, int bk, int64_t target, int min_chunks, int& splits,
                         int& kchunk) {
    int64_t want = ceil_div(target, std::max<int64_t>(tiles, 1));
    const int64_t maxs = std::max<int64_t>(1, K / (bk * min_chunks));
    want = std::min(want, maxs);
    if (want < 1) want = 1;
    kchunk = (int)(ceil_div(ceil_div(K, want), bk) * bk);
    splits = (int)ceil_div(K, kchunk);
}

struct Plan {
    Tile t;
    int splits, kchunk;
    int M, N, K;
};

// FWD/DGRAD: split K only when the output tiling leaves most CUs idle (the
// latency-bound tail of a round, when few clients are still training).
constexpr int kMnSplitBelow = 192;  // sweeps (fc_bench.py)
constexpr bool g_dgrad_s2_off = false;  // (r01 A/B switch, retired: phases always on)
constexpr int kMnTarget = 768;

static Plan plan_mn(int M, int N, int K, int nclients) {
    Plan p{pick_mn_tile(M, N), 1, K, M, N, K};
    const int64_t tiles = ceil_div(N, p.t.bn) * ceil_div(M, p.t.bm) * (int64_t)nclients;
    if (tiles < fill(kMnSplitBelow))
        choose_split(tiles, K, p.t.bk, fill(kMnTarget), 4, p.splits, p.kchunk);
    if (p.splits <= 1) {
        p.splits = 1;
        p.kchunk = K;
    }
    return p;
}

static Plan plan_wgrad(int M, int N, int K, int nclients) {
    Plan p{pick_wgrad_tile(M), 1, K, M, N, K};
    const int64_t tiles = ceil_div(N, p.t.bn) * ceil_div(M, p.t.bm) * (int64_t)nclients;
    choose_split(tiles, K, p.t.bk, fill(2048), 4, p.splits, p.kchunk);
    return p;
}

static size_t mn_ws_bytes(const Plan& p, int nclients) {
    return p.splits > 1 ? (size_t)nclients * p.splits * p.M * p.N * sizeof(float) : 0;
}

static size_t wgrad_ws_bytes(const Plan& p, int nclients) {
    if (p.splits == 1) return 0;  // written in place
    const size_t w = (size_t)nclients * p.splits * p.M * p.N * sizeof(float);
    const size_t b = (size_t)nclients * p.splits * p.M * sizeof(float);
    return ((w + 255) / 256) * 256 + b;
}

static int conv_common_check(int nclients, int batch, int cin, int h, int w, int cout, int kh,
                             int kw, int stride, int pad, int& oh, int& ow) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && cin > 0 && h > 0 && w > 0 && cout > 0,
               "conv: bad shape");
    FH_REQUIRE(stride > 0 && pad >= 0 && kh > 0 && kw > 0, "conv: bad kernel params");
    oh = (h + 2 * pad - kh) / stride + 1;
    ow = (w + 2 * pad - kw) / stride + 1;
    FH_REQUIRE(oh > 0 && ow > 0, "conv: empty output");
    FH_REQUIRE((int64_t)batch * std::max(oh * ow, h * w) < (1ll << 31), "conv: too many pixels");
    return FH_OK;
}

static ConvArgs make_args(int batch, int cin, int h, int w, int cout, int oh, int ow, int pad,
                          const int32_t* counts) {
    ConvArgs a{};
    a.batch = batch;
    a.cin = cin;
    a.h = h;
    a.w = w;
    a.cout = cout;
    a.oh = oh;
    a.ow = ow;
    a.pad = pad;
    a.counts = counts;
    a.splits = 1;
    a.fd_ohw = FastDiv(oh * ow);
    a.fd_ow = FastDiv(ow);
    a.fd_hw = FastDiv(h * w);
    a.fd_w = FastDiv(w);
    return a;
}

// Launch an FWD/DGRAD product, split-K through `ws` when the plan asks for it and
// the caller provided enough scratch; otherwise the single-pass kernel.
template <int OP>
static int run_mn(ConvArgs a, int kh, int kw, int stride, int nclients, void* ws, size_t ws_bytes,
                  float* out, int64_t out_cs, const float* bias, int64_t b_cs, int relu, int accum,
                  int sp, hipStream_t st, const char* name) {
    Plan p = plan_mn(a.M, a.N, a.K, nclients);
    if (p.splits > 1 && (!ws || ws_bytes < mn_ws_bytes(p, nclients))) {
        p.splits = 1;
        p.kchunk = a.K;
    }
    a.splits = p.splits;
    a.kchunk = p.kchunk;
    if (p.splits > 1) a.out = (float*)ws;
    dim3 grid((unsigned)ceil_div(a.N, p.t.bn), (unsigned)ceil_div(a.M, p.t.bm),
              (unsigned)(nclients * p.splits));
    int rc = launch_shape<OP>(kh, kw, stride, p.t, grid, a, st);
    if (rc) return rc;
    FH_LAUNCH_CHECK(name);
    if (p.splits > 1) {
        dim3 eg((unsigned)ceil_div(a.N, 256), (unsigned)a.M, (unsigned)nclients);
        FH_LAUNCH(splitk_epilogue_kernel, eg, dim3(256), 0, st, (const float*)ws, p.splits,
                           a.M, a.N, out, out_cs, bias, b_cs, relu, accum, a.counts, a.batch, sp,
                           (double*)nullptr, 0, a.drop, BnBwdEpi{}, PoolEpi{});
        FH_LAUNCH_CHECK(name);
    }
    return FH_OK;
}

// ---- stride-2 DGRAD by parity phases (OP_DGRAD_S2) -------------------------
static bool dgrad_s2_supported(int h, int w, int kh, int kw, int stride, int pad) {
    return stride == 2 && h % 2 == 0 && w % 2 == 0 &&
           ((kh == 3 && kw == 3 && pad == 1) || (kh == 1 && kw == 1 && pad == 0));
}

// W[z][co][ci][kh][kw] -> wp[z][phase][ci][co * taps + t] (igemm OP_DGRAD_S2's k order:
// t indexes the phase's taps, kh-major; 3x3/p1 phase (py, px) takes kh = 1 (py = 0) or
// {0, 2} (py = 1), likewise kw)
__global__ void __launch_bounds__(256)
pack_dgrad_s2_kernel(const float* __restrict__ w, int64_t w_cs, float* __restrict__ wp,
                     int64_t wp_cs, int cin, int cout, int KH) {
    const int z = blockIdx.y;
    const int KHW = KH * KH;
    const int64_t total = (int64_t)cin * cout * KHW;
    for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
        // phase of e: the prefix table over ci*cout-sized blocks
        const int blk = (int)(e / ((int64_t)cin * cout));
        int ph = 0;
        while (ph < 3 && s2_tap_prefix(KH, ph + 1) <= blk) ++ph;
        const int py = ph >> 1, px = ph & 1;
        const int nth = KH == 3 ? 1 + py : 1 - py, ntw = KH == 3 ? 1 + px : 1 - px;
        const int taps = nth * ntw;
        const int64_t r = e - (int64_t)s2_tap_prefix(KH, ph) * cin * cout;  // [ci][co*taps+t]
        const int ci = (int)(r / ((int64_t)cout * taps));
        const int k = (int)(r - (int64_t)ci * cout * taps);
        const int co = k / taps, t = k - co * taps;
        const int kh = KH == 3 ? (py ? 2 * (t / ntw) : 1) : 0;
        const int kw = KH == 3 ? (px ? 2 * (t % ntw) : 1) : 0;
        wp[z * wp_cs + e] = w[z * w_cs + ((int64_t)co * cin + ci) * KHW + kh * KH + kw];
    }
}

static size_t dgrad_s2_pack_bytes(int cin, int cout, int kh, int nclients) {
    return ((size_t)nclients * cin * cout * kh * kh * sizeof(float) + 255) / 256 * 256;
}
constexpr int g_dgrad_s2_pack = 1;  // A/B: 0 = gather W

// GEMM per (client, phase): M = cin, N = batch * oh * ow, K <= cout * 4 (3x3) or cout (1x1)
static Plan plan_dgrad_s2(int cin, int cout, int kh, int batch, int oh, int ow, int nclients) {
    return plan_mn(cin, batch * oh * ow, cout * (kh == 3 ? 4 : 1), nclients * 4);
}

static int run_dgrad_s2(ConvArgs a, int kh, int nclients, void* ws, size_t ws_bytes, float* out,
                        int64_t out_cs, int accum, hipStream_t st) {
    Plan p = plan_dgrad_s2(a.cin, a.cout, kh, a.batch, a.oh, a.ow, nclients);
    // workspace: [packed weights][split-K slab]; the pack goes first so that it survives
    // when the slab does not fit
    const size_t pack = g_dgrad_s2_pack ? dgrad_s2_pack_bytes(a.cin, a.cout, kh, nclients) : 0;
    if (pack && ws && ws_bytes >= pack) {
        a.wp = (float*)ws;
        a.wp_cs = (int64_t)a.cin * a.cout * kh * kh;
        FH_LAUNCH(pack_dgrad_s2_kernel,
                  dim3((unsigned)std::min<int64_t>(ceil_div(a.wp_cs, 256), 1024), nclients),
                  dim3(256), 0, st, a.wt, a.w_cs, (float*)ws, a.wp_cs, a.cin, a.cout, kh);
        FH_LAUNCH_CHECK("conv2d_dgrad s2 pack");
        ws = (char*)ws + pack;
        ws_bytes -= pack;
    }
    if (p.splits > 1 && (!ws || ws_bytes < mn_ws_bytes(p, nclients * 4))) {
        p.splits = 1;
        p.kchunk = p.K;
    }
    a.M = p.M;
    a.N = p.N;
    a.K = p.K;
    a.splits = p.splits;
    a.kchunk = p.kchunk;
    if (p.splits > 1) a.out = (float*)ws;
    dim3 grid((unsigned)ceil_div(a.N, p.t.bn), (unsigned)ceil_div(a.M, p.t.bm),
              (unsigned)(nclients * 4 * p.splits));
    int rc = launch_shape<OP_DGRAD_S2>(kh, kh, 2, p.t, grid, a, st);
    if (rc) return rc;
    FH_LAUNCH_CHECK("conv2d_dgrad s2");
    if (p.splits > 1) {
        dim3 eg((unsigned)ceil_div(a.N, 256), (unsigned)a.M, (unsigned)(nclients * 4));
        FH_LAUNCH(splitk_epilogue_s2_kernel, eg, dim3(256), 0, st, (const float*)ws, p.splits,
                  a.M, a.N, out, out_cs, accum, a.counts, a.batch, a.oh, a.ow, a.w);
        FH_LAUNCH_CHECK("conv2d_dgrad s2 epilogue");
    }
    return FH_OK;
}

// ---- direct 3x3 conv (dconv_kernels.h) planning ---------------------------
struct DPlan {
    int bm, ck, splits, cchunk;
};

static bool dconv_supported(int h, int w, int kh, int kw, int stride, int pad) {
    return kh == 3 && kw == 3 && stride == 1 && pad == 1 && h == w && (w == 8 || w == 16 || w == 32);
}

// Planner constants (MI355X sweeps: tools/conv_sweep.py on the CIFAR10CNN layers, r02 / r03
// A/B in profiles/): BM <= 64 once 512 workgroups are reached; the direct kernels split over
// input channels below 512 workgroups toward 1024, at most 4 splits (+0.5 % KT against no cap,
// r03 s4); stride-2 WGRAD 256 workgroups per resident wave; RGB-layer WGRAD 512 workgroups
// (42 -> 34 us at 32 clients, profiles/r01_v12).
constexpr int kDconvBlocks = 512;
constexpr int kDconvMaxBm = 64;
constexpr int kDwgradBlocks = 256;
constexpr int kDwgradSmallBlocks = 512;
constexpr int kDwgradMinSps = 1;
constexpr int kDconvSplitBelow = 512;
constexpr int kDconvSplitTarget = 1024;
constexpr int kDconvMaxSplits = 4;

static DPlan plan_dconv(int M, int Cr, int batch, int hw, int nclients, bool force_bm32 = false,
                        bool ck4 = false) {
    const int64_t tn = ceil_div((int64_t)batch * hw, 256);
    DPlan p{32, 8, 1, Cr};
    for (int bm : {128, 64}) {
        if (Cr <= 4 || force_bm32) break;  // tiny-Cin first layer / scalar staging: BM=32
        if (bm > kDconvMaxBm) continue;
        if (M >= bm && tn * ceil_div(M, bm) * nclients >= kDconvBlocks) {
            p.bm = bm;
            break;
        }
    }
    p.ck = (ck4 || p.bm == 128 || Cr <= 4) ? 4 : 8;
    const int64_t blocks = tn * ceil_div(M, p.bm) * nclients;
    const int chunks = (int)ceil_div(Cr, p.ck);
    if (blocks < fill(kDconvSplitBelow) && chunks > 1) {
        int want = (int)std::min<int64_t>(ceil_div(fill(kDconvSplitTarget), blocks), chunks);
        want = std::max(1, std::min(want, kDconvMaxSplits));
        const int per = (int)ceil_div(chunks, want);
        p.cchunk = per * p.ck;
        p.splits = (int)ceil_div(Cr, p.cchunk);
    }
    if (p.splits <= 1) {
        p.splits = 1;
        p.cchunk = Cr;
    }
    return p;
}

// split slab: [z][split][M][Nfull] (splitk_epilogue_kernel), sized over the padded tile grid
static size_t dconv_ws_bytes(const DPlan& p, int nclients, int M, int batch, int hw) {
    if (p.splits <= 1) return 0;
    const size_t mpad = (size_t)ceil_div(M, p.bm) * p.bm;
    const size_t npad = (size_t)ceil_div((int64_t)batch * hw, 256) * 256;
    return (size_t)nclients * p.splits * mpad * npad * sizeof(float);
}

template <int OP, int W, int S = 1, bool BNB = false>
static int dconv_launch_w(const DPlan& p, dim3 grid, const DConvArgs& a, hipStream_t st) {
#define FH_DC(BM, WMV, CK, VEC)                                                                 \
    if (p.bm == BM && p.ck == CK && (a.wvec != 0) == VEC) {                                     \
        FH_LAUNCH((dconv_kernel<OP, W, BM, WMV, CK, VEC, S, BNB>), grid, dim3(256), 0, st, a); \
        return FH_OK;                                                                           \
    }
    if constexpr (BNB && OP == OP_DGRAD) {  // BN-backward statistics epilogue (BM <= 64)
        FH_DC(32, 1, 8, true)
        FH_DC(32, 1, 4, true)
        FH_DC(64, 2, 8, true)
        FH_DC(32, 1, 8, false)
        FH_DC(32, 1, 4, false)
    } else if constexpr (S == 1) {
        FH_DC(32, 1, 8, true)
        FH_DC(32, 1, 4, true)
        FH_DC(64, 2, 8, true)
        FH_DC(128, 2, 4, true)
        FH_DC(32, 1, 8, false)
        FH_DC(32, 1, 4, false)
    } else {  // stride 2 (forward): CK = 4 keeps the 2*SEGR+1-row patch at two stages in LDS
        FH_DC(32, 1, 4, true)
        FH_DC(64, 2, 4, true)
        FH_DC(128, 2, 4, true)
        FH_DC(32, 1, 4, false)
    }
#undef FH_DC
    set_error("dconv: no instantiation bm=%d ck=%d s=%d", p.bm, p.ck, S);
    return FH_E_UNSUPPORTED;
}

// Dual-role layer backward (dconv_wgrad_dual_kernel).  fh_conv_pair(mode > 0) arms the next
// WGRAD on this thread: when it plans the quadrant-wave kernel with 128-pixel stages and its
// dW needs no reduction launch of its own (one split, or a deferred slab), the launch is held
// here and issued together with the next direct DGRAD on the same stream and map width
// (BM = 32, CK = 8 plan) as one grid.  Anything else flushes it as its own launch first;
// fh_conv_pair(0) flushes and disarms.  mode 1: WGRAD workgroups first, 2: DGRAD first.
struct PendingWgrad {
    bool on = false;
    int w = 0, mode = 1;
    bool pdy = false;  // its dY is the armed pooled gradient (g_pdy), not yet materialised
    dim3 grid;
    DWArgs d{};
    hipStream_t st = nullptr;
};
// r06 in-launch split-K reduction: the calling thread's ticket counters (zeroed once by the
// caller, left zero by every launch: each tile's last arriver resets its counter), one per
// output tile of a split direct FWD / DGRAD launch (fh_set_split_tickets)
struct SplitTickets {
    uint32_t* p = nullptr;
    int64_t n = 0;
};
thread_local SplitTickets g_tickets;
thread_local int64_t g_inl_launches = 0;  // fh_conv_pair_status-style instrumentation
thread_local int g_pair_mode = 0;
thread_local PendingWgrad g_pend;
thread_local int64_t g_dual_launches = 0;  // fh_conv_pair_status (instrumentation)
constexpr bool kDualForceBm32 = true;

// Pooled output gradient of the next WGRAD + DGRAD pair (fh_conv_pooled_dy, r05): when the pair
// becomes one dual-role launch on 16x16 planes, both roles route dY from the pooled gradient on
// load (PooledDy) and the dY tensor is never written; on any other path the pair's dY buffer is
// first filled by fh_maxpool2_bwd_ymask (the unfused step's own launch), once.
struct PdyArm {
    bool on = false, done = false;
    PooledDy p{};
};
thread_local PdyArm g_pdy;

// Deferred DGRAD reduction (fh_conv_defer_dgrad, r05): the next split direct DGRAD on 16x16
// planes with a plain sum epilogue leaves its partial slab unreduced; the conv1 weight gradient
// that reads its output (c1 pooled WGRAD, per-image slabs) sums the partials as it stages them,
// with the epilogue's order — one launch less per narrow step.  Anything else materialises it
// (the epilogue launch it skipped) first.
struct DgradDefer {
    bool armed = false, pending = false;
    const float* part = nullptr;
    int splits = 0, M = 0, nclients = 0, batch = 0;
    int64_t Nfull = 0, out_cs = 0;
    float* out = nullptr;
    const int32_t* counts = nullptr;
    hipStream_t st = nullptr;
};
thread_local DgradDefer g_ddef;
// instrumentation (fh_conv_defer_status): DGRADs left unreduced, and partial slabs a consumer
// summed while staging (the rest were materialised by the skipped epilogue launch)
thread_local int64_t g_ddef_deferred = 0, g_ddef_taken = 0;

// Split reduction left to the BatchNorm call after the conv (fh_conv_bn_defer, r06,
// splitbn.h): armed by the host for the next fh_conv2d_{fwd,dgrad}_bnstats call, recorded by
// run_dconv in place of its splitk_epilogue_kernel launch, consumed by the BN call (bn.hip);
// anything else that finds it pending launches the skipped epilogue (sbn_materialize).
thread_local SplitBnRec g_sbn;
thread_local int g_sbn_armed = 0;  // fh_conv_bn_defer(max) -> the next _bnstats call
thread_local int g_sbn_want = 0;   // ... inside that call
thread_local int64_t g_sbn_deferred = 0;

SplitBnRec& sbn_rec() { return g_sbn; }

int sbn_materialize() {
    if (!g_sbn.pending) return FH_OK;
    g_sbn.pending = false;
    const SplitBnRec& r = g_sbn;
    dim3 eg((unsigned)ceil_div(r.Nfull, 256), (unsigned)r.M, (unsigned)r.nclients);
    FH_LAUNCH(splitk_epilogue_kernel, eg, dim3(256), 0, r.st, r.part, r.splits, r.M, (int)r.Nfull,
              r.out, r.out_cs, r.bias, r.b_cs, 0, 0, r.counts, r.batch, r.sp, r.bn_part,
              r.bn_tiles, DropArgs{},
              BnBwdEpi{r.bnx, r.bnx_cs, r.bn_scale, r.bn_shift, r.bns_cs, r.bn_mean, r.pidx,
                       r.pmask, r.pi_cs, r.pm_cs, r.pscale, r.pw},
              PoolEpi{});
    FH_LAUNCH_CHECK("split conv reduction (deferred)");
    return FH_OK;
}

static int ddef_materialize() {
    if (!g_ddef.pending) return FH_OK;
    g_ddef.pending = false;
    const DgradDefer& d = g_ddef;
    dim3 eg((unsigned)ceil_div(d.Nfull, 256), (unsigned)d.M, (unsigned)d.nclients);
    FH_LAUNCH(splitk_epilogue_kernel, eg, dim3(256), 0, d.st, d.part, d.splits, d.M, (int)d.Nfull,
              d.out, d.out_cs, (const float*)nullptr, (int64_t)0, 0, 0, d.counts, d.batch, 256,
              (double*)nullptr, 0, DropArgs{}, BnBwdEpi{}, PoolEpi{});
    FH_LAUNCH_CHECK("deferred dgrad reduction");
    return FH_OK;
}

// the partials for a consumer reading `dpool` (planes of 256 pixels) on stream st, else {}
// after materialising whatever is pending
static int ddef_take(const float* dpool, int64_t dp_cs, int gh, int gw, hipStream_t st,
                     DgradParts& dp) {
    dp = DgradParts{};
    if (!g_ddef.pending) return FH_OK;
    if (g_ddef.out == dpool && g_ddef.out_cs == dp_cs && g_ddef.st == st && gh * gw == 256 &&
        g_ddef.splits <= kDgradPartsMax) {
        dp = DgradParts{g_ddef.part, g_ddef.splits, g_ddef.M, g_ddef.Nfull};
        g_ddef.pending = false;
        ++g_ddef_taken;
        return FH_OK;
    }
    return ddef_materialize();
}

static int pdy_materialize(float* dy, int64_t dy_cs, const int32_t* counts, int nclients,
                           int batch, int C, int plane, hipStream_t st) {
    if (!g_pdy.on || g_pdy.done) return FH_OK;
    g_pdy.done = true;
    const PooledDy& q = g_pdy.p;
    return fh_maxpool2_bwd_ymask(q.g, q.g_cs, q.idx, q.i_cs, q.yp, q.y_cs, dy, dy_cs, counts,
                                 nclients, batch, C, 2 * q.ph, 2 * q.ph, q.ph, q.ph, plane, plane,
                                 st);
}

static int flush_pending_wgrad() {
    if (!g_pend.on) return FH_OK;
    if (g_pend.pdy) {  // issued on its own: its dY must exist first
        g_pend.pdy = false;
        const int rc = pdy_materialize(const_cast<float*>(g_pend.d.dy), g_pend.d.dy_cs,
                                       g_pend.d.counts, (int)g_pend.grid.z, g_pend.d.batch,
                                       g_pend.d.M, g_pend.w, g_pend.st);
        if (rc) return rc;
    }
    g_pend.on = false;
    const PendingWgrad& q = g_pend;
    if (q.w == 32) FH_LAUNCH((dwgrad_q_kernel<32, 128, false>), q.grid, dim3(256), 0, q.st, q.d);
    else if (q.w == 16) FH_LAUNCH((dwgrad_q_kernel<16, 128, false>), q.grid, dim3(256), 0, q.st, q.d);
    else FH_LAUNCH((dwgrad_q_kernel<8, 128, false>), q.grid, dim3(256), 0, q.st, q.d);
    FH_LAUNCH_CHECK("conv2d_wgrad direct (held)");
    return FH_OK;
}

template <int W, bool BNB, bool PDY = false>
static int launch_dual(const DPlan& p, dim3 grid, const DConvArgs& a, hipStream_t st) {
    (void)p;
    const PendingWgrad& q = g_pend;
    const int64_t nw = (int64_t)q.grid.x * q.grid.y * q.grid.z;
    const int64_t nd = (int64_t)grid.x * grid.y * grid.z;
    FH_REQUIRE(nw + nd < (1ll << 31), "dual conv backward: grid %lld + %lld", (long long)nw,
               (long long)nd);
    FH_LAUNCH((dconv_wgrad_dual_kernel<W, BNB, PDY>), dim3((unsigned)(nw + nd)), dim3(256), 0,
              st, q.d, (int)q.grid.x, (int)q.grid.y, (int)nw, a, (int)grid.x, (int)grid.y,
              (int)nd, q.mode == 1 ? 1 : 0);
    ++g_dual_launches;
    return FH_OK;
}

template <int OP, int S = 1>
static int run_dconv(DConvArgs a, int w, int nclients, void* ws, size_t ws_bytes, int sp,
                     hipStream_t st, const char* name, bool* pooled = nullptr) {
    const int sbn_want = g_sbn_want;
    g_sbn_want = 0;
    if (const int rc = sbn_materialize()) return rc;  // a pending split output may be read here
    DPlan p = plan_dconv(a.M, a.Cr, a.batch, sp, nclients, false, S == 2);
    const bool aligned = ((uintptr_t)a.wt % 16 == 0) && a.w_cs % 4 == 0;
    if (!(aligned && (OP == OP_FWD ? a.Cr % p.ck == 0 : a.M % p.bm == 0)) && p.bm != 32) {
        p = plan_dconv(a.M, a.Cr, a.batch, sp, nclients, /*force_bm32=*/true, S == 2);  // scalar
    }
    if constexpr (OP == OP_DGRAD && S == 1) {
        // r05: a held WGRAD of this map width pairs only with a BM = 32 DGRAD — plan that
        // instead of BM = 64 so the layer's backward stays one dual-role launch on wide grids
        // (KT conv4 and the ResNet 64-channel layers at >= 16 clients ran as two launches)
        if (kDualForceBm32 && g_pend.on && g_pend.st == st && g_pend.w == w && p.bm != 32)
            p = plan_dconv(a.M, a.Cr, a.batch, sp, nclients, /*force_bm32=*/true, false);
    }
    if (p.splits > 1 && (!ws || ws_bytes < dconv_ws_bytes(p, nclients, a.M, a.batch, sp))) {
        p.splits = 1;
        p.cchunk = a.Cr;
    }
    a.splits = p.splits;
    a.cchunk = p.cchunk;
    a.Nfull = a.batch * sp;
    dim3 grid((unsigned)ceil_div(a.Nfull, 256), (unsigned)ceil_div(a.M, p.bm),
              (unsigned)(nclients * p.splits));
    // r06: a split plan reduces in-launch (the tile's last arriver, dconv_body) when the
    // thread has ticket counters for its tiles — except a DGRAD the deferred reduction will
    // leave to conv1's weight gradient (fh_conv_defer_dgrad: its consumer reads the
    // splitk_epilogue slab layout)
    bool inl = p.splits > 1 && g_tickets.p != nullptr &&
               (int64_t)grid.x * grid.y * nclients <= g_tickets.n;
    if constexpr (OP == OP_DGRAD && S == 1) {
        if (inl && g_ddef.armed && w == 16 && !a.accumulate && a.bnx == nullptr &&
            a.pidx == nullptr && p.splits <= kDgradPartsMax)
            inl = false;
    }
    // split launches pool in the split reduction when each of its workgroups holds one whole
    // image plane (sp = 256), else in a separate pass after it (the caller); an in-launch
    // reduction pools in its last arriver's epilogue
    if (p.splits > 1 && sp != 256 && !inl) a.pool_y = nullptr;
    if (pooled) *pooled = a.pool_y != nullptr;
    // float4 weight runs: 16-B aligned slices that never run past the tensor
    a.wvec = aligned && (OP == OP_FWD ? a.Cr % p.ck == 0 : a.M % p.bm == 0);
    float* out = a.out;
    if (inl) {
        a.slab = (float*)ws;
        a.tickets = g_tickets.p;
        a.gx = (int)grid.x;
        a.gy = (int)grid.y;
        ++g_inl_launches;
    } else if (p.splits > 1) {
        a.out = (float*)ws;
    }
    int rc;
    bool dual = false;
    if constexpr (OP == OP_DGRAD && S == 1) {
        if (g_pend.on) {
            if (g_pend.st == st && g_pend.w == w && p.bm == 32 && p.ck == 8 && a.wvec) {
                const bool bnb = a.bn_part && (p.splits == 1 || inl);
                if (g_pend.pdy && w == 16 && !bnb && !a.accumulate) {
                    // the pooled gradient routed on load by both roles: dY is never written
                    a.pdy = g_pdy.p;
                    g_pdy.done = true;
                    rc = launch_dual<16, false, true>(p, grid, a, st);
                } else {
                    if (g_pend.pdy) {
                        g_pend.pdy = false;
                        rc = pdy_materialize(const_cast<float*>(a.in), a.in_cs, a.counts, nclients,
                                             a.batch, a.Cr, w, st);
                        if (rc) return rc;
                    }
                    rc = w == 32 ? (bnb ? launch_dual<32, true>(p, grid, a, st)
                                        : launch_dual<32, false>(p, grid, a, st))
                       : w == 16 ? (bnb ? launch_dual<16, true>(p, grid, a, st)
                                        : launch_dual<16, false>(p, grid, a, st))
                                 : (bnb ? launch_dual<8, true>(p, grid, a, st)
                                        : launch_dual<8, false>(p, grid, a, st));
                }
                g_pend.on = false;
                g_pend.pdy = false;
                if (rc) return rc;
                dual = true;
            } else if (const int fr = flush_pending_wgrad()) {
                return fr;
            }
        }
        if (!dual && g_pdy.on && !g_pdy.done) {  // this DGRAD reads the pair's dY: fill it
            rc = pdy_materialize(const_cast<float*>(a.in), a.in_cs, a.counts, nclients, a.batch,
                                 a.Cr, w, st);
            if (rc) return rc;
        }
    }
    if (dual) {
        rc = FH_OK;
    } else if constexpr (S == 2) {
        rc = w == 16 ? dconv_launch_w<OP, 16, 2>(p, grid, a, st)
                     : dconv_launch_w<OP, 8, 2>(p, grid, a, st);
    } else if ((a.bn_part || (a.pool_y && p.bm != 32)) && (p.splits == 1 || inl)) {
        // the statistics-epilogue instances (and the pooled epilogue at BM = 64, whose tile
        // image needs their LDS; at BM = 32 the plain instance pools in the K loop's LDS)
        rc = w == 32 ? dconv_launch_w<OP, 32, 1, true>(p, grid, a, st)
           : w == 16 ? dconv_launch_w<OP, 16, 1, true>(p, grid, a, st)
                     : dconv_launch_w<OP, 8, 1, true>(p, grid, a, st);
    } else {
        rc = w == 32 ? dconv_launch_w<OP, 32>(p, grid, a, st)
           : w == 16 ? dconv_launch_w<OP, 16>(p, grid, a, st)
                     : dconv_launch_w<OP, 8>(p, grid, a, st);
    }
    if (rc) return rc;
    FH_LAUNCH_CHECK(name);
    if constexpr (OP == OP_DGRAD && S == 1) {
        if (g_ddef.armed) {
            g_ddef.armed = false;  // the next DGRAD only
            if (!inl && p.splits > 1 && w == 16 && !a.accumulate && a.bnx == nullptr &&
                a.pidx == nullptr && p.splits <= kDgradPartsMax) {
                if (const int rc = ddef_materialize()) return rc;
                g_ddef.pending = true;
                g_ddef.part = (const float*)ws;
                g_ddef.splits = p.splits;
                g_ddef.M = a.M;
                g_ddef.Nfull = a.Nfull;
                g_ddef.out = out;
                g_ddef.out_cs = a.out_cs;
                g_ddef.counts = a.counts;
                g_ddef.nclients = nclients;
                g_ddef.batch = a.batch;
                g_ddef.st = st;
                ++g_ddef_deferred;
                return FH_OK;
            }
        }
    }
    if (p.splits > 1 && !inl) {
        if (sbn_want && S == 1 && a.bn_part && !a.accumulate && !a.relu && !a.pool_y &&
            p.splits <= 4 && (int64_t)a.batch * sp <= std::min(sbn_want, kSbnMaxElems) &&
            a.bn_tiles == ceil_div(a.Nfull, 256) &&
            (OP == OP_FWD ? a.bnx == nullptr : a.bnx != nullptr)) {
            // the BN call after this conv sums the slab (splitbn.h, fh_conv_bn_defer)
            SplitBnRec& r = g_sbn;
            r = SplitBnRec{};
            r.op = OP == OP_FWD ? 0 : 1;
            r.part = (const float*)ws;
            r.splits = p.splits; r.M = a.M; r.sp = sp; r.batch = a.batch; r.nclients = nclients;
            r.Nfull = a.Nfull;
            r.out = out; r.out_cs = a.out_cs;
            r.bias = OP == OP_FWD ? a.bias : nullptr; r.b_cs = a.b_cs;
            r.counts = a.counts;
            r.bn_part = a.bn_part; r.bn_tiles = a.bn_tiles;
            if (OP != OP_FWD) {
                r.bnx = a.bnx; r.bnx_cs = a.bnx_cs; r.bn_scale = a.bn_scale;
                r.bn_shift = a.bn_shift; r.bns_cs = a.bns_cs; r.bn_mean = a.bn_mean;
                r.pidx = a.pidx; r.pmask = a.pmask; r.pi_cs = a.pi_cs; r.pm_cs = a.pm_cs;
                r.pscale = a.pscale; r.pw = w;
            }
            r.st = st;
            r.pending = true;
            ++g_sbn_deferred;
            return FH_OK;
        }
        dim3 eg((unsigned)ceil_div(a.Nfull, 256), (unsigned)a.M, (unsigned)nclients);
        FH_LAUNCH(splitk_epilogue_kernel, eg, dim3(256), 0, st, (const float*)ws, p.splits,
                           a.M, a.Nfull, out, a.out_cs, OP == OP_FWD ? a.bias : nullptr, a.b_cs,
                           OP == OP_FWD ? a.relu : 0, OP == OP_FWD ? 0 : a.accumulate, a.counts,
                           a.batch, sp, a.bn_part, a.bn_tiles, DropArgs{},
                           BnBwdEpi{OP == OP_FWD ? nullptr : a.bnx, a.bnx_cs, a.bn_scale,
                                    a.bn_shift, a.bns_cs, a.bn_mean, a.pidx, a.pmask, a.pi_cs,
                                    a.pm_cs, a.pscale, w},
                           PoolEpi{OP == OP_FWD ? a.pool_y : nullptr, a.pool_idx, a.py_cs,
                                   a.pix_cs, a.pool_hw, w});
        FH_LAUNCH_CHECK(name);
    }
    return FH_OK;
}

// 3x3 / stride 2 / pad 1 forward on square maps with an 8x8 or 16x16 output (ResNet
// down-sampling blocks, 32->16 and 16->8): dconv_kernel<FWD, W_out, ..., S=2>
constexpr bool g_dconv_s2_off = false;  // A/B: back to igemm
static bool dconv_s2_supported(int h, int w, int kh, int kw, int stride, int pad) {
    return !g_dconv_s2_off && kh == 3 && kw == 3 && stride == 2 && pad == 1 && h == w &&
           (w == 16 || w == 32);
}

// 3x3 / stride 2 / pad 1 DGRAD on square 32->16 and 16->8 maps (ResNet down-sampling blocks):
// dconv_dgrad_s2_kernel<grid width, CK = 8>, 32 dX channels per workgroup, split over the
// reduction channels (cout) on small grids.
constexpr bool g_dconv_dgrad_s2_off = false;
static bool dconv_dgrad_s2_supported(int h, int w, int kh, int kw, int stride, int pad, int cin,
                                     int cout) {
    return !g_dconv_dgrad_s2_off && kh == 3 && kw == 3 && stride == 2 && pad == 1 && h == w &&
           (w == 16 || w == 32) && cin % 32 == 0 && cout % 8 == 0;
}
// split planning (sweeps): target workgroups (two fit a CU) and the fewest reduction channels a
// split keeps (every split writes a slab the size of dX: few long splits beat many short ones)
constexpr int kDs2Fill = 256;
constexpr int kDs2MinCh = 32;
static DPlan plan_dconv_dgrad_s2(int cin, int cout, int batch, int oh, int nclients) {
    DPlan p{32, 8, 1, cout};
    const int64_t blocks = ceil_div((int64_t)batch * oh * oh, 256) * ceil_div(cin, 32) * nclients;
    const int chunks = (int)ceil_div(cout, 8);
    const int maxs = std::max(1, (int)(cout / std::max(8, kDs2MinCh)));
    if (blocks < fill(kDs2Fill) && chunks > 1) {
        const int want = (int)std::min<int64_t>(ceil_div(fill(kDs2Fill), blocks), maxs);
        const int per = (int)ceil_div(chunks, std::max(1, want));
        p.cchunk = per * 8;
        p.splits = (int)ceil_div(cout, p.cchunk);
    }
    if (p.splits <= 1) {
        p.splits = 1;
        p.cchunk = cout;
    }
    return p;
}
static int run_dconv_dgrad_s2(DConvArgs a, int oh, int nclients, void* ws, size_t ws_bytes,
                              hipStream_t st) {
    const bool sc = a.in2 != nullptr;
    const int sp = 4 * oh * oh;  // dX pixels per image
    DPlan p = plan_dconv_dgrad_s2(a.M, a.Cr, a.batch, oh, nclients);
    if (p.splits > 1 && (!ws || ws_bytes < dconv_ws_bytes(p, nclients, a.M, a.batch, sp))) {
        p.splits = 1;
        p.cchunk = a.Cr;
    }
    a.splits = p.splits;
    a.cchunk = p.cchunk;
    a.Nfull = a.batch * sp;
    float* out = a.out;
    if (p.splits > 1) a.out = (float*)ws;
    dim3 grid((unsigned)ceil_div((int64_t)a.batch * oh * oh, 256), (unsigned)ceil_div(a.M, 32),
              (unsigned)(nclients * p.splits));
    if (oh == 16 && sc) {
        FH_LAUNCH((dconv_dgrad_s2_kernel<16, 8, true>), grid, dim3(256), 0, st, a);
    } else if (oh == 16) {
        FH_LAUNCH((dconv_dgrad_s2_kernel<16, 8, false>), grid, dim3(256), 0, st, a);
    } else if (sc) {
        FH_LAUNCH((dconv_dgrad_s2_kernel<8, 8, true>), grid, dim3(256), 0, st, a);
    } else {
        FH_LAUNCH((dconv_dgrad_s2_kernel<8, 8, false>), grid, dim3(256), 0, st, a);
    }
    FH_LAUNCH_CHECK("conv2d_dgrad direct s2");
    if (p.splits > 1) {
        dim3 eg((unsigned)ceil_div(a.Nfull, 256), (unsigned)a.M, (unsigned)nclients);
        FH_LAUNCH(splitk_epilogue_kernel, eg, dim3(256), 0, st, (const float*)ws, p.splits, a.M,
                  a.Nfull, out, a.out_cs, nullptr, (int64_t)0, 0, a.accumulate, a.counts, a.batch,
                  sp, nullptr, 0, DropArgs{}, BnBwdEpi{}, PoolEpi{});
        FH_LAUNCH_CHECK("conv2d_dgrad direct s2 epilogue");
    }
    return FH_OK;
}

// 1x1 / stride 2 / pad 0 forward on square 32->16 and 16->8 maps (the ResNet projection
// shortcut): pw_s2_fwd_kernel<output width, CK = 16>
constexpr bool g_pw_s2_off = false;
static bool pw_s2_supported(int h, int w, int kh, int kw, int stride, int pad, int cin) {
    return !g_pw_s2_off && kh == 1 && kw == 1 && stride == 2 && pad == 0 && h == w &&
           (w == 16 || w == 32) && cin % 16 == 0;
}

// ---- direct 3x3 wgrad planning -------------------------------------------
struct DWPlan {
    int wco, wci, wpx, sr, splits, sps;
};

static bool dwgrad_supported(int cin, int cout, int h, int w, int kh, int kw, int stride, int pad) {
    return dconv_supported(h, w, kh, kw, stride, pad) && cin % 32 == 0 && cout % 32 == 0;
}

// r03 quadrant-wave WGRAD (dconv_kernels.h dwgrad_q_kernel): 32x32 (co, ci) tiles, 128-pixel
// stages, three 45 KB workgroups per CU; splits of the stage run fill ~kDwqBlocks workgroups
// (512: tools/r03_wgrad_ab.sh sweep, profiles/r03_dwq/).  KT against the r02 kernel (32x32x2
// MFMAs, four pixel-waves, one 86 KB workgroup per CU): 270.3k / 272.1k vs 269.3k / 269.2k
// client-images/s, interleaved.
constexpr int kDwqBlocks = 1024;
// stage pixels: 128 = one buffer, stored between two barriers; the 64-pixel double-buffered
// instance (the next stage stored half-way through this one's MFMAs) measured within noise of
// it (profiles/r03_dwq/) and serves the per-image DP-SGD slabs of 8x8 maps (one image a stage)
constexpr int kDwqSpx = 128;
static DWPlan plan_dwq(int cout, int cin, int batch, int w, int nclients) {
    DWPlan p{1, 1, 4, kDwqSpx / w, 1, 1};
    const int64_t tiles = (int64_t)(cout / 32) * (cin / 32) * nclients;
    const int nst = (int)ceil_div((int64_t)batch * w * w, (int64_t)kDwqSpx);
    const int want = (int)std::min<int64_t>(std::max<int64_t>(1, ceil_div(fill(kDwqBlocks), tiles)),
                                            std::max(1, nst / kDwgradMinSps));
    p.sps = (int)ceil_div(nst, want);
    p.splits = (int)ceil_div(nst, p.sps);
    return p;
}

// RGB first layer (cin == 3): (ci,kh,kw) = 27 on the MFMA lanes, pixels split 4 ways
static bool dwgrad_small_supported(int cin, int cout, int h, int w, int kh, int kw, int stride,
                                   int pad) {
    return dconv_supported(h, w, kh, kw, stride, pad) && cin == 3 && cout % 32 == 0;
}

static DWPlan plan_dwgrad_small(int cout, int batch, int w, int nclients) {
    DWPlan p{1, 1, 4, 128 / w, 1, 1};
    const int64_t tiles = (int64_t)(cout / 32) * nclients;
    const int nst = (int)ceil_div((int64_t)batch * w * w, (int64_t)p.sr * w);
    const int want = (int)std::min<int64_t>(
        std::max<int64_t>(1, ceil_div(fill(kDwgradSmallBlocks), tiles)),
        std::max(1, nst / kDwgradMinSps));
    p.sps = (int)ceil_div(nst, want);
    p.splits = (int)ceil_div(nst, p.sps);
    return p;
}

// 3x3 / stride 2 / pad 1 WGRAD on square 32->16 / 16->8 maps (ResNet down-sampling blocks):
// dconv_wgrad_kernel<output width, WCO = 2, WCI = 1, WPX = 2, 64-pixel stages, S = 2> — 64 x 32
// (co, ci) tiles, so each staged input patch (2*SEGR+1 rows) feeds twice the MFMAs;
constexpr bool g_dwgrad_s2_off = false;
static bool dwgrad_s2_supported(int cin, int cout, int h, int w, int kh, int kw, int stride,
                                int pad) {
    return !g_dwgrad_s2_off && kh == 3 && kw == 3 && stride == 2 && pad == 1 && h == w &&
           (w == 16 || w == 32) && cin % 32 == 0 && cout % 64 == 0;
}
static DWPlan plan_dwgrad_s2(int cout, int cin, int batch, int wo, int nclients) {
    DWPlan p{2, 1, 2, 64 / wo, 1, 1};
    const int64_t tiles = (int64_t)(cout / 64) * (cin / 32) * nclients;
    const int nst = (int)ceil_div((int64_t)batch * wo * wo, (int64_t)p.sr * wo);
    const int occ = dwgrad_occ(wo, 2, 1, p.sr, 2);
    const int want = (int)std::min<int64_t>(
        std::max<int64_t>(1, ceil_div(fill(kDwgradBlocks * occ), tiles)),
        std::max(1, nst / kDwgradMinSps));
    p.sps = (int)ceil_div(nst, want);
    p.splits = (int)ceil_div(nst, p.sps);
    return p;
}

// single-input-channel 3x3 / s1 / p1 (SimpleCNN conv1): conv_c1_fwd_kernel / conv_c1_wgrad_kernel;
constexpr bool g_conv_c1_off = false;
static bool conv_c1_supported(int cin, int cout, int kh, int kw, int stride, int pad) {
    return !g_conv_c1_off && cin == 1 && kh == 3 && kw == 3 && stride == 1 && pad == 1 &&
           (cout == 32 || cout == 64);
}
static int conv_c1_chunks(int batch, int h, int w) {
    return (int)ceil_div((int64_t)batch * h * w, kC1Chunk);
}
// conv1 WGRAD on the matrix cores (conv_c1_wgrad_mfma_kernel): 4-row stages, ~kC1MfmaBlocks
// workgroups (the kernel is HBM-bound: many small workgroups keep loads in flight)
constexpr int kC1MfmaBlocks = 1024;
constexpr int kC1MinSps = 2;  // stages per chunk at least
static bool conv_c1_mfma_ok(int h, int w) { return h % 4 == 0 && w % 4 == 0 && w <= 32; }
static DWPlan plan_c1_mfma(int batch, int h, int nclients) {
    const int nst = batch * (h / 4);
    int want = (int)std::max<int64_t>(1, ceil_div(fill(kC1MfmaBlocks), std::max(nclients, 1)));
    want = std::min(want, std::max(1, nst / std::max(1, kC1MinSps)));
    DWPlan p{1, 1, 1, 4, 1, 1};
    p.sps = (int)ceil_div(nst, want);
    p.splits = (int)ceil_div(nst, p.sps);
    return p;
}

// byte offset of the bias partials behind the weight partials [client][split][MN] of a
// WGRAD slab (every WGRAD path lays its workspace out this way)
static int64_t wslab_bias_off(int nclients, int splits, int64_t MN) {
    return (int64_t)(((size_t)nclients * splits * MN * sizeof(float) + 255) / 256 * 256);
}

static size_t dwgrad_ws_bytes(const DWPlan& p, int nclients, int M, int N) {
    const size_t wb = (size_t)nclients * p.splits * M * N * sizeof(float);
    return ((wb + 255) / 256) * 256 + (size_t)nclients * p.splits * M * sizeof(float);
}

}  // namespace fh

using namespace fh;

extern "C" int fh_set_fill_fraction(float fraction) {
    FH_REQUIRE(fraction > 0.f && fraction <= 1.f, "fill fraction must be in (0, 1]");
    g_fill = fraction;
    return FH_OK;
}

extern "C" float fh_get_fill_fraction(void) { return g_fill; }

extern "C" int fh_conv_pair(int32_t mode) {
    FH_REQUIRE(mode >= -1 && mode <= 2, "conv_pair: mode %d", mode);
    if (mode < 0) {  // error paths: drop a held launch unissued
        g_pair_mode = 0;
        g_pend.on = false;
        g_pend.pdy = false;
        g_pdy = PdyArm{};
        // ... and a deferred DGRAD reduction armed or left pending by the failed step: its
        // partials would otherwise be claimed (or never reduced) by an unrelated later launch
        g_ddef = DgradDefer{};
        g_sbn = SplitBnRec{};  // likewise a split reduction left for a BN call
        g_sbn_armed = 0;
        return FH_OK;
    }
    if (mode > 0) {
        g_pair_mode = mode;
        return FH_OK;
    }
    g_pair_mode = 0;
    const int rc = flush_pending_wgrad();
    g_pdy = PdyArm{};
    return rc;
}

// fh_conv_defer_dgrad(1): the calling thread's next split direct DGRAD on 16x16 planes with a
// plain sum epilogue leaves its partials unreduced for the conv1 weight gradient that reads its
// output (fh_conv2d_c1_pool_wgrad[_deferred], fh_conv2d_c1_pool_wgrad_persample[_clip]), which
// sums them as it stages them — the epilogue's order, the same bits (r05).  A consumer of any
// other tensor, or fh_conv_defer_dgrad(0), launches the skipped reduction first.
extern "C" int fh_conv_defer_dgrad(int32_t on) {
    g_ddef.armed = on != 0;
    if (!on) return ddef_materialize();
    return FH_OK;
}

// r06: ticket counters for the calling thread's in-launch split-K reductions (direct 3x3
// stride-1 FWD / DGRAD with a split plan, incl. the dual-role DGRAD): n uint32 words the caller
// zeroed once and keeps alive while any launch (or captured step) that used them may run; each
// launch leaves them zero.  p = NULL: split plans launch splitk_epilogue_kernel as before.
extern "C" int fh_set_split_tickets(void* p, int64_t n) {
    FH_REQUIRE((p == nullptr) == (n == 0) && n >= 0 && ((uintptr_t)p % 4) == 0,
               "set_split_tickets: bad buffer");
    g_tickets = SplitTickets{(uint32_t*)p, n};
    return FH_OK;
}

extern "C" int fh_split_tickets_status(int64_t* inl_launches) {
    FH_REQUIRE(inl_launches, "split_tickets_status: null pointer");
    *inl_launches = g_inl_launches;
    return FH_OK;
}

// fh_conv_bn_defer(1): the calling thread's next fh_conv2d_fwd_bnstats /
// fh_conv2d_dgrad_bnstats call, when it plans a split direct launch, leaves its split reduction
// to the BatchNorm call that consumes its statistics (fh_bn_finalize_tiles,
// fh_maxpool2_fwd_bnfinalize, fh_bn_bwd_tiles, fh_bn_bwd_pool_tiles), which then sums the slab
// and runs the BN pass as one launch — bit-identical outputs (splitbn.h).  A DGRAD's stored
// gradient (dX) is then never written: only that BN call reads it.  Any other library call
// that finds the reduction pending launches it first.  max_elems: the largest batch x plane
// (elements per client and channel, <= 8192) the fusion takes; 0 disarms.
extern "C" int fh_conv_bn_defer(int32_t max_elems) {
    FH_REQUIRE(max_elems >= 0, "conv_bn_defer: %d", max_elems);
    g_sbn_armed = max_elems;
    return FH_OK;
}

extern "C" int fh_conv_bn_defer_status(int64_t* deferred, int64_t* taken) {
    FH_REQUIRE(deferred && taken, "conv_bn_defer_status: null pointer");
    *deferred = g_sbn_deferred;
    *taken = sbn_taken();
    return FH_OK;
}

extern "C" int fh_conv_defer_status(int64_t* deferred, int64_t* taken) {
    FH_REQUIRE(deferred && taken, "conv_defer_status: null pointer");
    *deferred = g_ddef_deferred;
    *taken = g_ddef_taken;
    return FH_OK;
}

extern "C" int fh_conv_pooled_dy(const float* dpool, int64_t dp_cs, const uint8_t* pidx,
                                 int64_t pi_cs, const float* ypool, int64_t yp_cs, int32_t ph) {
    FH_REQUIRE(dpool && pidx && ypool && ph > 0, "conv_pooled_dy: bad arguments");
    g_pdy.on = true;
    g_pdy.done = false;
    g_pdy.p = PooledDy{dpool, pidx, ypool, dp_cs, pi_cs, yp_cs, ph};
    return FH_OK;
}

extern "C" int fh_launch_ts_set(void* rec, void* count, uint32_t cap, int32_t w, int32_t cin,
                                int32_t cout) {
    FH_REQUIRE(!rec || (count && cap > 0 && ((uintptr_t)rec % 16) == 0 && w > 0 && cin > 0 &&
                        cout > 0 && cin < 4096 && cout < 4096 && w < 256),
               "launch_ts_set: bad arguments");
    LaunchTs t{(uint32_t*)rec, (uint32_t*)count, rec ? cap : 0u,
               rec ? dual_shape_key(w, cin, cout) : 0u};
    const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_launch_ts), &t, sizeof(t));
    FH_REQUIRE(e == hipSuccess, "launch_ts_set: %s", hipGetErrorString(e));
    return FH_OK;
}

extern "C" int fh_wall_clock_khz(int32_t* khz) {
    FH_REQUIRE(khz, "wall_clock_khz: null pointer");
    int dev = 0, v = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev);
    FH_REQUIRE(e == hipSuccess, "wall_clock_khz: %s", hipGetErrorString(e));
    *khz = v;
    return FH_OK;
}

extern "C" int fh_conv_pair_status(int32_t* held, int64_t* dual_launches) {
    FH_REQUIRE(held && dual_launches, "conv_pair_status: null pointer");
    *held = g_pend.on ? 1 : 0;
    *dual_launches = g_dual_launches;
    return FH_OK;
}

extern "C" size_t fh_conv2d_fwd_workspace(int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                                          int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                                          int32_t stride, int32_t pad) {
    int oh = (h + 2 * pad - kh) / stride + 1, ow = (w_ + 2 * pad - kw) / stride + 1;
    if (oh <= 0 || ow <= 0 || nclients <= 0) return 0;
    if (dconv_supported(h, w_, kh, kw, stride, pad))
        return dconv_ws_bytes(plan_dconv(cout, cin, batch, h * w_, nclients), nclients, cout, batch,
                              h * w_);
    if (dconv_s2_supported(h, w_, kh, kw, stride, pad)) {
        size_t b = dconv_ws_bytes(plan_dconv(cout, cin, batch, oh * ow, nclients, false, true),
                                  nclients, cout, batch, oh * ow);
        size_t b32 = dconv_ws_bytes(plan_dconv(cout, cin, batch, oh * ow, nclients, true, true),
                                    nclients, cout, batch, oh * ow);  // scalar-staging plan
        return b > b32 ? b : b32;
    }
    return mn_ws_bytes(plan_mn(cout, batch * oh * ow, cin * kh * kw, nclients), nclients);
}

extern "C" size_t fh_conv2d_dgrad_workspace(int32_t nclients, int32_t batch, int32_t cin,
                                            int32_t h, int32_t w_, int32_t cout, int32_t kh,
                                            int32_t kw, int32_t stride, int32_t pad) {
    int oh = (h + 2 * pad - kh) / stride + 1, ow = (w_ + 2 * pad - kw) / stride + 1;
    if (oh <= 0 || ow <= 0 || nclients <= 0) return 0;
    if (dconv_supported(h, w_, kh, kw, stride, pad))
        return dconv_ws_bytes(plan_dconv(cin, cout, batch, h * w_, nclients), nclients, cin, batch,
                              h * w_);
    size_t direct_s2 = 0;
    if (dconv_dgrad_s2_supported(h, w_, kh, kw, stride, pad, cin, cout))
        direct_s2 = dconv_ws_bytes(plan_dconv_dgrad_s2(cin, cout, batch, oh, nclients), nclients,
                                   cin, batch, h * w_);
    if (dgrad_s2_supported(h, w_, kh, kw, stride, pad) && !g_dgrad_s2_off)
        return std::max(direct_s2,
                        (g_dgrad_s2_pack ? dgrad_s2_pack_bytes(cin, cout, kh, nclients) : 0) +
                            mn_ws_bytes(plan_dgrad_s2(cin, cout, kh, batch, oh, ow, nclients),
                                        nclients * 4));
    return std::max(direct_s2,
                    mn_ws_bytes(plan_mn(cin, batch * h * w_, cout * kh * kw, nclients), nclients));
}

static int conv2d_fwd_impl(const float* x, int64_t x_cs, const float* in_scale,
                           const float* in_shift, int64_t aff_cs, const float* w, int64_t w_cs,
                           const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                           const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin,
                           int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                           int32_t stride, int32_t pad, int32_t relu, void* workspace,
                           size_t ws_bytes, void* stream, double* bn_part = nullptr) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && w && y, "conv2d_fwd: null pointer");
    FH_REQUIRE((in_scale == nullptr) == (in_shift == nullptr), "conv2d_fwd: scale/shift pair");
    if (dconv_supported(h, w_, kh, kw, stride, pad)) {
        DConvArgs d{};
        d.in = x; d.wt = w; d.bias = bias; d.out = y;
        d.in_cs = x_cs; d.w_cs = w_cs; d.b_cs = b_cs; d.out_cs = y_cs;
        d.counts = counts; d.batch = batch; d.Cr = cin; d.M = cout; d.relu = relu;
        d.in_scale = in_scale; d.in_shift = in_shift; d.aff_cs = aff_cs;
        d.bn_part = bn_part; d.bn_tiles = (int)ceil_div((int64_t)batch * h * w_, 256);
        return run_dconv<OP_FWD>(d, w_, nclients, workspace, ws_bytes, h * w_, as_stream(stream),
                                 "conv2d_fwd");
    }
    if (!in_scale && !bn_part && conv_c1_supported(cin, cout, kh, kw, stride, pad)) {
        dim3 grid((unsigned)ceil_div((int64_t)batch * h * w_, 256), (unsigned)nclients);
        hipStream_t st = as_stream(stream);
        if (cout == 32)
            FH_LAUNCH(conv_c1_fwd_kernel<32>, grid, dim3(256), 0, st, x, x_cs, w, w_cs, bias,
                      b_cs, y, y_cs, counts, batch, h, w_, relu);
        else
            FH_LAUNCH(conv_c1_fwd_kernel<64>, grid, dim3(256), 0, st, x, x_cs, w, w_cs, bias,
                      b_cs, y, y_cs, counts, batch, h, w_, relu);
        FH_LAUNCH_CHECK("conv2d_fwd c1");
        return FH_OK;
    }
    if (!in_scale && !bn_part && dconv_s2_supported(h, w_, kh, kw, stride, pad)) {
        DConvArgs d{};
        d.in = x; d.wt = w; d.bias = bias; d.out = y;
        d.in_cs = x_cs; d.w_cs = w_cs; d.b_cs = b_cs; d.out_cs = y_cs;
        d.counts = counts; d.batch = batch; d.Cr = cin; d.M = cout; d.relu = relu;
        return run_dconv<OP_FWD, 2>(d, ow, nclients, workspace, ws_bytes, oh * ow,
                                    as_stream(stream), "conv2d_fwd_s2");
    }
    if (!in_scale && !bn_part && pw_s2_supported(h, w_, kh, kw, stride, pad, cin) &&
        (uintptr_t)x % 16 == 0 && x_cs % 4 == 0 && (uintptr_t)w % 16 == 0 && w_cs % 4 == 0) {
        DConvArgs d{};
        d.in = x; d.wt = w; d.bias = bias; d.out = y;
        d.in_cs = x_cs; d.w_cs = w_cs; d.b_cs = b_cs; d.out_cs = y_cs;
        d.counts = counts; d.batch = batch; d.Cr = cin; d.M = cout; d.relu = relu;
        dim3 grid((unsigned)ceil_div((int64_t)batch * oh * ow, 256), (unsigned)ceil_div(cout, 64),
                  (unsigned)nclients);
        hipStream_t st = as_stream(stream);
        if (ow == 16) FH_LAUNCH((pw_s2_fwd_kernel<16, 16>), grid, dim3(256), 0, st, d);
        else FH_LAUNCH((pw_s2_fwd_kernel<8, 16>), grid, dim3(256), 0, st, d);
        FH_LAUNCH_CHECK("conv2d_fwd 1x1 s2");
        return FH_OK;
    }
    if (in_scale || bn_part) {
        set_error("conv2d_fwd_bnrelu / _bnstats: need the direct 3x3 path (3x3/s1/p1, square "
                  "8/16/32)");
        return FH_E_UNSUPPORTED;
    }
    ConvArgs a = make_args(batch, cin, h, w_, cout, oh, ow, pad, counts);
    a.x = x; a.wt = w; a.bias = bias; a.out = y;
    a.x_cs = x_cs; a.w_cs = w_cs; a.b_cs = b_cs; a.out_cs = y_cs;
    a.relu = relu;
    a.M = cout; a.N = batch * oh * ow; a.K = cin * kh * kw;
    return run_mn<OP_FWD>(a, kh, kw, stride, nclients, workspace, ws_bytes, y, y_cs, bias, b_cs,
                          relu, 0, oh * ow, as_stream(stream), "conv2d_fwd");
}

extern "C" int fh_conv2d_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                             const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                             const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin,
                             int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                             int32_t stride, int32_t pad, int32_t relu, void* workspace,
                             size_t ws_bytes, void* stream) {
    return conv2d_fwd_impl(x, x_cs, nullptr, nullptr, 0, w, w_cs, bias, b_cs, y, y_cs, counts,
                           nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, relu, workspace,
                           ws_bytes, stream);
}

extern "C" int fh_conv2d_fwd_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                                    const float* in_shift, int64_t aff_cs, const float* w,
                                    int64_t w_cs, const float* bias, int64_t b_cs, float* y,
                                    int64_t y_cs, const int32_t* counts, int32_t nclients,
                                    int32_t batch, int32_t cin, int32_t h, int32_t w_,
                                    int32_t cout, int32_t kh, int32_t kw, int32_t stride,
                                    int32_t pad, int32_t relu, void* workspace, size_t ws_bytes,
                                    void* stream) {
    FH_REQUIRE(in_scale && in_shift, "conv2d_fwd_bnrelu: null scale/shift");
    return conv2d_fwd_impl(x, x_cs, in_scale, in_shift, aff_cs, w, w_cs, bias, b_cs, y, y_cs,
                           counts, nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, relu,
                           workspace, ws_bytes, stream);
}

// BatchNorm partial statistics of a direct-conv FWD output: bytes of the fp64 (sum, sum of
// squares) pairs per (client, channel, 256-pixel tile) that fh_conv2d_fwd_bnstats writes.
extern "C" size_t fh_conv_bnstats_bytes(int32_t nclients, int32_t batch, int32_t cout, int32_t h,
                                        int32_t w_) {
    if (nclients <= 0 || batch <= 0 || cout <= 0 || h <= 0 || w_ <= 0) return 0;
    return (size_t)nclients * cout * ceil_div((int64_t)batch * h * w_, 256) * 2 * sizeof(double);
}

// fh_conv2d_fwd_bnrelu (in_scale / in_shift nullable) that also leaves the BatchNorm
// statistics of y in bn_part (fh_conv_bnstats_bytes; merged by fh_bn_finalize_tiles), so the
// BN layer after this conv never re-reads y.  Direct 3x3 path only; no ReLU on y.
extern "C" int fh_conv2d_fwd_bnstats(const float* x, int64_t x_cs, const float* in_scale,
                                     const float* in_shift, int64_t aff_cs, const float* w,
                                     int64_t w_cs, const float* bias, int64_t b_cs, float* y,
                                     int64_t y_cs, double* bn_part, const int32_t* counts,
                                     int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                                     int32_t w_, int32_t cout, void* workspace, size_t ws_bytes,
                                     void* stream) {
    FH_REQUIRE(bn_part, "conv2d_fwd_bnstats: null statistics buffer");
    FH_REQUIRE(dconv_supported(h, w_, 3, 3, 1, 1), "conv2d_fwd_bnstats: needs a 3x3/s1/p1 conv "
               "on a square 8/16/32 map (got %dx%d)", h, w_);
    g_sbn_want = g_sbn_armed;
    g_sbn_armed = 0;
    const int rc = conv2d_fwd_impl(x, x_cs, in_scale, in_shift, aff_cs, w, w_cs, bias, b_cs, y,
                                   y_cs, counts, nclients, batch, cin, h, w_, cout, 3, 3, 1, 1, 0,
                                   workspace, ws_bytes, stream, bn_part);
    g_sbn_want = 0;
    return rc;
}

extern "C" int fh_maxpool2_fwd_pitched(const float* x, int64_t x_cs, float* y, int64_t y_cs,
                                       uint8_t* idx, int64_t i_cs, uint8_t* mask, int64_t m_cs,
                                       const int32_t* counts, int32_t nclients, int32_t batch,
                                       int32_t C, int32_t H, int32_t W, int32_t drop_mode,
                                       float p_drop, uint64_t seed, const uint64_t* seed_dev,
                                       int32_t xh, int32_t xw, int32_t yh, int32_t yw,
                                       void* stream);  // layers.hip

// conv (3x3 / s1 / p1) -> ReLU -> 2x2 max-pool of the top-left pool_hw x pool_hw map of each
// h x w plane (SimpleCNN conv2 + pool2, models_pytorch.py:88-89, on 16x16 planes holding the
// 14x14 map).  py / pidx: dense [img][cout][pool_hw/2][pool_hw/2] (maxpool2_fwd_kernel's values
// and first-max argmax, bit for bit).  Unsplit launches pool in the conv's epilogue, split
// launches on 16x16 planes in the split reduction (splitk_epilogue_kernel, PoolEpi), neither
// writes y; split launches on 8x8 planes write y (scratch) and pool it in a separate pass.  The
// pool's backward therefore takes its ReLU mask from py (fh_maxpool2_bwd_ymask): the pooled
// value IS the ReLU output at the argmax.
extern "C" int fh_conv2d_fwd_relu_pool(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                                       const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                                       float* py, int64_t py_cs, uint8_t* pidx, int64_t pi_cs,
                                       const int32_t* counts, int32_t nclients, int32_t batch,
                                       int32_t cin, int32_t h, int32_t w_, int32_t cout,
                                       int32_t pool_hw, void* workspace, size_t ws_bytes,
                                       void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, 3, 3, 1, 1, oh, ow);
    if (rc) return rc;
    FH_REQUIRE(dconv_supported(h, w_, 3, 3, 1, 1) && h <= 16, "conv2d_fwd_relu_pool: needs a "
               "square 8 or 16 map (whole images per 256-pixel tile), got %dx%d", h, w_);
    FH_REQUIRE(pool_hw >= 2 && pool_hw <= h && !(pool_hw & 1), "conv2d_fwd_relu_pool: pooled "
               "map %d in a %d plane", pool_hw, h);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && w && y && py && pidx, "conv2d_fwd_relu_pool: null pointer");
    DConvArgs d{};
    d.in = x; d.wt = w; d.bias = bias; d.out = y;
    d.in_cs = x_cs; d.w_cs = w_cs; d.b_cs = b_cs; d.out_cs = y_cs;
    d.counts = counts; d.batch = batch; d.Cr = cin; d.M = cout; d.relu = 1;
    d.pool_y = py; d.pool_idx = pidx; d.py_cs = py_cs; d.pix_cs = pi_cs; d.pool_hw = pool_hw;
    bool fused = false;
    rc = run_dconv<OP_FWD>(d, w_, nclients, workspace, ws_bytes, h * w_, as_stream(stream),
                           "conv2d_fwd_relu_pool", &fused);
    if (rc || fused) return rc;
    return fh_maxpool2_fwd_pitched(y, y_cs, py, py_cs, pidx, pi_cs, nullptr, 0, counts, nclients,
                                   batch, cout, pool_hw, pool_hw, 0, 0.f, 0, nullptr, h, w_,
                                   pool_hw / 2, pool_hw / 2, stream);
}

extern "C" int fh_conv2d_dgrad(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs,
                               float* dx, int64_t dx_cs, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t cin, int32_t h, int32_t w_, int32_t cout,
                               int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                               int32_t accumulate, void* workspace, size_t ws_bytes,
                               void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && w && dx, "conv2d_dgrad: null pointer");
    if (dconv_supported(h, w_, kh, kw, stride, pad)) {
        DConvArgs d{};
        d.in = dy; d.wt = w; d.out = dx;
        d.in_cs = dy_cs; d.w_cs = w_cs; d.out_cs = dx_cs;
        d.counts = counts; d.batch = batch; d.Cr = cout; d.M = cin; d.accumulate = accumulate;
        return run_dconv<OP_DGRAD>(d, w_, nclients, workspace, ws_bytes, h * w_, as_stream(stream),
                                   "conv2d_dgrad");
    }
    if (dconv_dgrad_s2_supported(h, w_, kh, kw, stride, pad, cin, cout) &&
        (uintptr_t)w % 16 == 0 && w_cs % 4 == 0 && (uintptr_t)dx % 8 == 0 && dx_cs % 2 == 0) {
        DConvArgs d{};
        d.in = dy; d.wt = w; d.out = dx;
        d.in_cs = dy_cs; d.w_cs = w_cs; d.out_cs = dx_cs;
        d.counts = counts; d.batch = batch; d.Cr = cout; d.M = cin; d.accumulate = accumulate;
        return run_dconv_dgrad_s2(d, oh, nclients, workspace, ws_bytes, as_stream(stream));
    }
    ConvArgs a = make_args(batch, cin, h, w_, cout, oh, ow, pad, counts);
    a.dy = dy; a.wt = w; a.out = dx;
    a.dy_cs = dy_cs; a.w_cs = w_cs; a.out_cs = dx_cs;
    a.accumulate = accumulate;
    if (dgrad_s2_supported(h, w_, kh, kw, stride, pad) && !g_dgrad_s2_off)
        return run_dgrad_s2(a, kh, nclients, workspace, ws_bytes, dx, dx_cs, accumulate,
                            as_stream(stream));
    a.M = cin; a.N = batch * h * w_; a.K = cout * kh * kw;
    return run_mn<OP_DGRAD>(a, kh, kw, stride, nclients, workspace, ws_bytes, dx, dx_cs, nullptr, 0,
                            0, accumulate, h * w_, as_stream(stream), "conv2d_dgrad");
}

// fh_conv2d_dgrad (3x3/s1/p1 direct path) whose input was relu(BN(bn_x)) — CIFAR10CNN
// bn1/bn3/bn5 (models_pytorch.py:133-150): stores the ReLU-masked gradient
// g = (bn_x*scale + shift > 0) ? dX : 0 (scale / shift: that BN's affine, fh_bn_fwd_stats /
// fh_bn_finalize_tiles) and leaves the BN backward statistics (sum g, sum (bn_x - mean) g) in
// bn_part (fh_conv_bnstats_bytes layout), so fh_bn_bwd_tiles replaces fh_bn_bwd's reduce
// pass over g and bn_x.  pidx non-null: relu(BN(bn_x)) went through MaxPool2d(2,2) (+ the
// Dropout after it: pmask / p_drop, as fh_bn_bwd_pool) first — bn2/bn4 (:139-150); bn_x is
// the 2h x 2w map, dX is stored unmasked and the statistics route it to the window argmax
// (fh_bn_bwd_pool_tiles is then the apply pass).
extern "C" int fh_conv2d_dgrad_bnstats(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs,
                                       float* dx, int64_t dx_cs, const float* bn_x,
                                       int64_t bnx_cs, const float* bn_scale,
                                       const float* bn_shift, int64_t bns_cs,
                                       const float* bn_mean, double* bn_part,
                                       const uint8_t* pidx, int64_t pi_cs, const uint8_t* pmask,
                                       int64_t pm_cs, float p_drop,
                                       const int32_t* counts, int32_t nclients, int32_t batch,
                                       int32_t cin, int32_t h, int32_t w_, int32_t cout,
                                       void* workspace, size_t ws_bytes, void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, 3, 3, 1, 1, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && w && dx && bn_x && bn_scale && bn_shift && bn_mean && bn_part,
               "conv2d_dgrad_bnstats: null pointer");
    FH_REQUIRE(dconv_supported(h, w_, 3, 3, 1, 1), "conv2d_dgrad_bnstats: needs the direct 3x3 "
               "path (square 8/16/32 map, got %dx%d)", h, w_);
    DConvArgs d{};
    d.in = dy; d.wt = w; d.out = dx;
    d.in_cs = dy_cs; d.w_cs = w_cs; d.out_cs = dx_cs;
    d.counts = counts; d.batch = batch; d.Cr = cout; d.M = cin;
    d.bn_part = bn_part; d.bn_tiles = (int)ceil_div((int64_t)batch * h * w_, 256);
    d.bnx = bn_x; d.bnx_cs = bnx_cs; d.bn_scale = bn_scale; d.bn_shift = bn_shift;
    d.bns_cs = bns_cs; d.bn_mean = bn_mean;
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "conv2d_dgrad_bnstats: p=%g", p_drop);
    d.pidx = pidx; d.pmask = pidx ? pmask : nullptr; d.pi_cs = pi_cs; d.pm_cs = pm_cs;
    d.pscale = 1.0f / (1.0f - p_drop);
    g_sbn_want = g_sbn_armed;
    g_sbn_armed = 0;
    rc = run_dconv<OP_DGRAD>(d, w_, nclients, workspace, ws_bytes, h * w_, as_stream(stream),
                             "conv2d_dgrad_bnstats");
    g_sbn_want = 0;
    return rc;
}

// The DGRAD of a ResNet down-sampling block's input in one launch (models_pytorch.py:176-194:
// conv1 3x3 / stride 2 / pad 1 and the 1x1 / stride-2 projection shortcut read the same
// input): dx (=|+=) dgrad3x3(dy, w) + dgrad1x1s2(dy_sc, w_sc).  dy_sc has dy's shape, w_sc is
// [cout][cin] per client.  Direct stride-2 kernel only (square 32 / 16 maps, cin % 32 == 0,
// cout % 8 == 0, 16-B aligned weights, 8-B aligned dx rows): FH_E_UNSUPPORTED otherwise.
// Workspace: fh_conv2d_dgrad_workspace of the 3x3 conv.
extern "C" int fh_conv2d_dgrad_s2_shortcut(const float* dy, int64_t dy_cs, const float* w,
                                           int64_t w_cs, const float* dy_sc, int64_t dysc_cs,
                                           const float* w_sc, int64_t wsc_cs, float* dx,
                                           int64_t dx_cs, const int32_t* counts,
                                           int32_t nclients, int32_t batch, int32_t cin,
                                           int32_t h, int32_t w_, int32_t cout,
                                           int32_t accumulate, void* workspace, size_t ws_bytes,
                                           void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, 3, 3, 2, 1, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && w && dy_sc && w_sc && dx, "conv2d_dgrad_s2_shortcut: null pointer");
    if (!(dconv_dgrad_s2_supported(h, w_, 3, 3, 2, 1, cin, cout) && (uintptr_t)w % 16 == 0 &&
          w_cs % 4 == 0 && (uintptr_t)dx % 8 == 0 && dx_cs % 2 == 0 &&
          (uintptr_t)dy_sc % 16 == 0 && dysc_cs % 4 == 0)) {
        set_error("conv2d_dgrad_s2_shortcut: outside the direct stride-2 kernel (%dx%d, cin %d, "
                  "cout %d)", h, w_, cin, cout);
        return FH_E_UNSUPPORTED;
    }
    DConvArgs d{};
    d.in = dy; d.wt = w; d.out = dx;
    d.in_cs = dy_cs; d.w_cs = w_cs; d.out_cs = dx_cs;
    d.in2 = dy_sc; d.wt2 = w_sc; d.in2_cs = dysc_cs; d.w2_cs = wsc_cs;
    d.counts = counts; d.batch = batch; d.Cr = cout; d.M = cin; d.accumulate = accumulate;
    return run_dconv_dgrad_s2(d, oh, nclients, workspace, ws_bytes, as_stream(stream));
}

namespace fh {
static int conv_c1_pool_launch(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                               const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                               uint8_t* idx, int64_t i_cs, const int32_t* counts, int nclients,
                               int batch, int h, int w_, int cout, int yh, int yw, const U8Src& src,
                               hipStream_t st) {
    const bool wide = nclients >= kC1PoolWide;
    const int cg = wide ? cout : 8;
    dim3 grid((unsigned)ceil_div((int64_t)batch * (h / 2) * (w_ / 2), 256), (unsigned)(cout / cg),
              (unsigned)nclients);
#define FH_C1P(CO, CG)                                                                           \
    FH_LAUNCH((conv_c1_pool_fwd_kernel<CO, CG>), grid, dim3(256), 0, st, x, x_cs, w, w_cs, bias,    \
              b_cs, y, y_cs, idx, i_cs, counts, batch, h, w_, yh, yw, src)
    if (cout == 32) {
        if (wide) FH_C1P(32, 32); else FH_C1P(32, 8);
    } else {
        if (wide) FH_C1P(64, 64); else FH_C1P(64, 8);
    }
#undef FH_C1P
    FH_LAUNCH_CHECK("conv2d_c1_pool_fwd");
    return FH_OK;
}
}  // namespace fh

// SimpleCNN conv1 -> ReLU -> 2x2 max-pool in one launch (conv_c1_pool_fwd_kernel): y = the
// pooled output in planes yh x yw (the H/2 x W/2 map in the top-left corner; yh = H/2, yw = W/2
// for dense planes), idx the dense uint8 argmax [img][cout][H/2][W/2].  cin = 1, 3x3 / s1 /
// p1, cout 32 or 64; the same values as fh_conv2d_fwd(relu) + fh_maxpool2_fwd.
extern "C" int fh_conv2d_c1_pool_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                                     const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                                     uint8_t* idx, int64_t i_cs, const int32_t* counts,
                                     int32_t nclients, int32_t batch, int32_t h, int32_t w_,
                                     int32_t cout, int32_t yh, int32_t yw, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && h >= 2 && w_ >= 2 && !(h & 1) && !(w_ & 1) &&
               yh >= h / 2 && yw >= w_ / 2, "conv2d_c1_pool_fwd: bad shape");
    FH_REQUIRE(cout == 32 || cout == 64, "conv2d_c1_pool_fwd: cout %d (32 or 64)", cout);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && w && y && idx, "conv2d_c1_pool_fwd: null pointer");
    return conv_c1_pool_launch(x, x_cs, w, w_cs, bias, b_cs, y, y_cs, idx, i_cs, counts, nclients,
                               batch, h, w_, cout, yh, yw, U8Src{}, as_stream(stream));
}

// fh_conv2d_c1_pool_fwd with the step's batch gather folded in (U8Src): x [z][batch][h][w] is
// WRITTEN from the raw uint8 images data[gidx[z][b]] ([N][h][w], one channel) with
// fh_gather_u8's normalisation (no crop / flip), and y_lab[z][b] = labels[gidx[z][b]] — the
// same x / labels fh_gather_u8 would leave, bit for bit, and the same pooled output.
extern "C" int fh_conv2d_c1_pool_fwd_u8(const uint8_t* data, const int64_t* labels,
                                        const int64_t* gidx, int64_t g_cs, float mean, float stdv,
                                        float* x, int64_t x_cs, int64_t* y_lab, int64_t yl_cs,
                                        const float* w, int64_t w_cs, const float* bias,
                                        int64_t b_cs, float* y, int64_t y_cs, uint8_t* idx,
                                        int64_t i_cs, const int32_t* counts, int32_t nclients,
                                        int32_t batch, int32_t h, int32_t w_, int32_t cout,
                                        int32_t yh, int32_t yw, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && h >= 2 && w_ >= 2 && !(h & 1) && !(w_ & 1) &&
               yh >= h / 2 && yw >= w_ / 2, "conv2d_c1_pool_fwd_u8: bad shape");
    FH_REQUIRE(cout == 32 || cout == 64, "conv2d_c1_pool_fwd_u8: cout %d (32 or 64)", cout);
    FH_REQUIRE(stdv != 0.f, "conv2d_c1_pool_fwd_u8: zero std");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(data && labels && gidx && x && y_lab && w && y && idx,
               "conv2d_c1_pool_fwd_u8: null pointer");
    const U8Src src{data, labels, gidx, g_cs, y_lab, yl_cs, mean, stdv, x, x_cs};
    return conv_c1_pool_launch(x, x_cs, w, w_cs, bias, b_cs, y, y_cs, idx, i_cs, counts, nclients,
                               batch, h, w_, cout, yh, yw, src, as_stream(stream));
}

// Its backward's weight gradient: fh_maxpool2_bwd(dpool, idx, xin = the ReLU output) +
// fh_conv2d_wgrad in one pass — the full-resolution gradient is never written; dpool and y
// (the pooled ReLU output, whose sign is the mask at the argmax) in planes gh x gw.
// Workspace: fh_conv2d_wgrad_workspace(nclients, batch, 1, h, w, cout, 3, 3, 1, 1).
static int c1_pool_wgrad_impl(const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs,
                              const uint8_t* idx, int64_t i_cs, const float* y, int64_t y_cs,
                              float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* workspace,
                              size_t ws_bytes, const int32_t* counts, int32_t nclients,
                              int32_t batch, int32_t h, int32_t w_, int32_t cout, int32_t gh,
                              int32_t gw, void* stream, int32_t* defer_splits,
                              int64_t* defer_boff) {
    // defer_splits: the partials left in the slab (>= 1; the optimizer sums them), 0 = dW / db
    // written directly (r06: single-split slab paths reported 1, which read as "direct", and the
    // layer's gradient never reached the optimizer)
    if (defer_splits) *defer_splits = 0;
    if (defer_boff) *defer_boff = 0;
    FH_REQUIRE(nclients >= 0 && batch > 0 && h >= 2 && w_ >= 2 && !(h & 1) && !(w_ & 1) &&
               gh >= h / 2 && gw >= w_ / 2, "conv2d_c1_pool_wgrad: bad shape");
    FH_REQUIRE(cout == 32 || cout == 64, "conv2d_c1_pool_wgrad: cout %d (32 or 64)", cout);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dpool && idx && y && dw, "conv2d_c1_pool_wgrad: null pointer");
    const bool mfma = conv_c1_mfma_ok(h, w_) && (uintptr_t)x % 16 == 0 && x_cs % 4 == 0;
    DWPlan p{1, 1, 1, 1, conv_c1_chunks(batch, h, w_), 1};
    if (mfma) p = plan_c1_mfma(batch, h, nclients);
    const size_t need = dwgrad_ws_bytes(p, nclients, cout, 9);
    FH_REQUIRE(workspace && ws_bytes >= need, "conv2d_c1_pool_wgrad: workspace %zu < %zu",
               ws_bytes, need);
    float* part = (float*)workspace;
    const size_t wbytes = ((size_t)nclients * p.splits * cout * 9 * sizeof(float) + 255) / 256 * 256;
    float* bpart = db ? (float*)((char*)workspace + wbytes) : nullptr;
    hipStream_t st = as_stream(stream);
    // a deferred DGRAD reduction of dpool (fh_conv_defer_dgrad): summed while staging, unless
    // this launch's own partial output would overlap the slab being read
    DgradParts dpa{};
    if (const int rc = ddef_take(dpool, dp_cs, gh, gw, st, dpa)) return rc;
    if (dpa.p && (!mfma || cout != 32 ||
                  ((const char*)dpa.p < (const char*)workspace + need &&
                   (const char*)workspace <
                       (const char*)(dpa.p + (int64_t)nclients * dpa.splits * dpa.M * dpa.Nfull)))) {
        g_ddef.pending = true;  // give it back and reduce it the usual way
        if (const int rc = ddef_materialize()) return rc;
        dpa = DgradParts{};
    }
    if (mfma) {  // conv_c1_wgrad_mfma_kernel<POOLED>: the routed gradient on the matrix cores
        const dim3 grid((unsigned)p.splits, (unsigned)nclients);
        if (cout == 32 && dpa.p)
            FH_LAUNCH((conv_c1_wgrad_mfma_kernel<32, true, 2, false, kDgradPartsMax>), grid,
                      dim3(256), 0, st, x, x_cs, dpool, dp_cs, part, bpart, counts, batch, h, w_,
                      p.splits, p.sps, idx, i_cs, y, y_cs, gh, gw, NormTail{}, dpa);
        else if (cout == 32)
            FH_LAUNCH((conv_c1_wgrad_mfma_kernel<32, true>), grid, dim3(256), 0, st, x, x_cs, dpool,
                      dp_cs, part, bpart, counts, batch, h, w_, p.splits, p.sps, idx, i_cs, y,
                      y_cs, gh, gw, NormTail{}, DgradParts{});
        else
            FH_LAUNCH((conv_c1_wgrad_mfma_kernel<64, true>), grid, dim3(256), 0, st, x, x_cs, dpool,
                      dp_cs, part, bpart, counts, batch, h, w_, p.splits, p.sps, idx, i_cs, y,
                      y_cs, gh, gw, NormTail{}, DgradParts{});
        FH_LAUNCH_CHECK("conv2d_c1_pool_wgrad mfma");
        if (defer_splits) {  // the optimizer step sums the chunks (fh_sgd_step_slabs)
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * 9);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)part, dw, dw_cs, p.splits, cout * 9,
                                      (const float*)bpart, db, db_cs, cout, nclients, st))
            return _r;
        FH_LAUNCH_CHECK("conv2d_c1_pool_wgrad reduce");
        return FH_OK;
    }
    FH_LAUNCH(conv_c1_wgrad_kernel<true>, dim3((unsigned)p.splits, (unsigned)(cout / 8), nclients),
              dim3(256), 0, st, x, x_cs, dpool, dp_cs, part, bpart, counts, batch, h, w_, cout,
              p.splits, idx, i_cs, y, y_cs, gh, gw);
    FH_LAUNCH_CHECK("conv2d_c1_pool_wgrad");
    const int MN = cout * 9;
    if (defer_splits) {
        *defer_splits = p.splits;
        *defer_boff = wslab_bias_off(nclients, p.splits, MN);
        return FH_OK;
    }
    if (const int _r = splitk_sum((const float*)part, dw, dw_cs, p.splits, MN, (const float*)bpart, db, db_cs, cout, nclients, st)) return _r;
    FH_LAUNCH_CHECK("conv2d_c1_pool_wgrad reduce");
    return FH_OK;
}

extern "C" int fh_conv2d_c1_pool_wgrad(const float* x, int64_t x_cs, const float* dpool,
                                       int64_t dp_cs, const uint8_t* idx, int64_t i_cs,
                                       const float* y, int64_t y_cs, float* dw, int64_t dw_cs,
                                       float* db, int64_t db_cs, void* workspace,
                                       size_t ws_bytes, const int32_t* counts, int32_t nclients,
                                       int32_t batch, int32_t h, int32_t w_, int32_t cout,
                                       int32_t gh, int32_t gw, void* stream) {
    return c1_pool_wgrad_impl(x, x_cs, dpool, dp_cs, idx, i_cs, y, y_cs, dw, dw_cs, db, db_cs,
                              workspace, ws_bytes, counts, nclients, batch, h, w_, cout, gh, gw,
                              stream, nullptr, nullptr);
}

extern "C" int fh_conv2d_c1_pool_wgrad_deferred(
    const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs, const uint8_t* idx,
    int64_t i_cs, const float* y, int64_t y_cs, float* dw, int64_t dw_cs, float* db, int64_t db_cs,
    void* slab, size_t slab_bytes, const int32_t* counts, int32_t nclients, int32_t batch,
    int32_t h, int32_t w_, int32_t cout, int32_t gh, int32_t gw, int32_t* splits_out,
    int64_t* bias_off_out, void* stream) {
    FH_REQUIRE(splits_out && bias_off_out, "conv2d_c1_pool_wgrad_deferred: null output");
    return c1_pool_wgrad_impl(x, x_cs, dpool, dp_cs, idx, i_cs, y, y_cs, dw, dw_cs, db, db_cs, slab,
                              slab_bytes, counts, nclients, batch, h, w_, cout, gh, gw, stream,
                              splits_out, bias_off_out);
}

extern "C" size_t fh_conv2d_wgrad_workspace(int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                                            int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                                            int32_t stride, int32_t pad) {
    int oh = (h + 2 * pad - kh) / stride + 1, ow = (w_ + 2 * pad - kw) / stride + 1;
    if (oh <= 0 || ow <= 0 || nclients <= 0) return 0;
    size_t direct = 0;
    if (dwgrad_supported(cin, cout, h, w_, kh, kw, stride, pad))  // (misaligned data: igemm)
        direct = dwgrad_ws_bytes(plan_dwq(cout, cin, batch, w_, nclients), nclients, cout,
                                 cin * 9);
    if (dwgrad_small_supported(cin, cout, h, w_, kh, kw, stride, pad))
        direct = dwgrad_ws_bytes(plan_dwgrad_small(cout, batch, w_, nclients), nclients, cout, cin * 9);
    if (dwgrad_s2_supported(cin, cout, h, w_, kh, kw, stride, pad))
        direct = dwgrad_ws_bytes(plan_dwgrad_s2(cout, cin, batch, ow, nclients), nclients, cout,
                                 cin * 9);
    if (conv_c1_supported(cin, cout, kh, kw, stride, pad)) {
        DWPlan p{1, 1, 1, 1, conv_c1_chunks(batch, h, w_), 1};  // (also the fused-pool form)
        direct = dwgrad_ws_bytes(p, nclients, cout, 9);
        if (conv_c1_mfma_ok(h, w_))
            direct = std::max(direct, dwgrad_ws_bytes(plan_c1_mfma(batch, h, nclients), nclients,
                                                      cout, 9));
    }
    return std::max(direct, wgrad_ws_bytes(plan_wgrad(cout, cin * kh * kw, batch * oh * ow, nclients),
                                           nclients));
}

static int conv2d_wgrad_impl(const float* x, int64_t x_cs, const float* in_scale,
                             const float* in_shift, int64_t aff_cs, const float* dy,
                             int64_t dy_cs, float* dw, int64_t dw_cs, float* db, int64_t db_cs,
                             void* workspace, size_t ws_bytes, const int32_t* counts,
                             int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w_,
                             int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                             void* stream, int32_t* defer_splits = nullptr,
                             int64_t* defer_boff = nullptr) {
    // defer_splits (fh_conv2d_wgrad_deferred): a split plan leaves its partials in the
    // workspace for the optimizer step to sum; the reduction launch is skipped
    const int pair = g_pair_mode;  // fh_conv_pair arms one call
    g_pair_mode = 0;
    // defer_splits: partials left in the slab (>= 1, also for a one-split plan whose kernel
    // writes the slab: c1, small-cin, stride 2), 0 = dW / db written directly
    if (defer_splits) *defer_splits = 0;
    if (defer_boff) *defer_boff = 0;
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && dw, "conv2d_wgrad: null pointer");
    FH_REQUIRE((in_scale == nullptr) == (in_shift == nullptr), "conv2d_wgrad: scale/shift pair");
    ConvArgs a = make_args(batch, cin, h, w_, cout, oh, ow, pad, counts);
    a.x = x; a.dy = dy;
    a.x_cs = x_cs; a.dy_cs = dy_cs;
    a.M = cout; a.N = cin * kh * kw; a.K = batch * oh * ow;
    const bool aligned = ((uintptr_t)x % 16 == 0) && ((uintptr_t)dy % 16 == 0) && x_cs % 4 == 0 &&
                         dy_cs % 4 == 0;
    // an armed pooled dY (fh_conv_pooled_dy) travels with a held 16x16 launch into the dual-role
    // grid; any other path reads dy, which is filled first
    bool pdy_hold = false;
    if (g_pdy.on && !g_pdy.done) {
        if (pair && !in_scale && aligned && w_ == 16 &&
            dwgrad_supported(cin, cout, h, w_, kh, kw, stride, pad)) {
            const DWPlan pq = plan_dwq(cout, cin, batch, w_, nclients);
            pdy_hold = pq.sr * w_ != 64 && (pq.splits == 1 || defer_splits);
        }
        if (!pdy_hold) {
            rc = pdy_materialize(const_cast<float*>(dy), dy_cs, counts, nclients, batch, cout, w_,
                                 as_stream(stream));
            if (rc) return rc;
        }
    }
    if (in_scale && !(aligned && dwgrad_supported(cin, cout, h, w_, kh, kw, stride, pad))) {
        set_error("conv2d_wgrad_bnrelu: needs the direct 3x3 wgrad (16-B aligned, channels %% 32)");
        return FH_E_UNSUPPORTED;
    }
    if (!in_scale && conv_c1_supported(cin, cout, kh, kw, stride, pad) && conv_c1_mfma_ok(h, w_) &&
        ((uintptr_t)x % 16 == 0) && ((uintptr_t)dy % 16 == 0) && x_cs % 4 == 0 && dy_cs % 4 == 0) {
        const DWPlan p = plan_c1_mfma(batch, h, nclients);
        const size_t need = dwgrad_ws_bytes(p, nclients, cout, 9);
        FH_REQUIRE(workspace && ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes,
                   need);
        float* part = (float*)workspace;
        const size_t wbytes = ((size_t)nclients * p.splits * cout * 9 * sizeof(float) + 255) / 256 * 256;
        float* bpart = db ? (float*)((char*)workspace + wbytes) : nullptr;
        hipStream_t st = as_stream(stream);
        const dim3 grid((unsigned)p.splits, (unsigned)nclients);
        if (cout == 32)
            FH_LAUNCH((conv_c1_wgrad_mfma_kernel<32, false>), grid, dim3(256), 0, st, x, x_cs, dy,
                      dy_cs, part, bpart, counts, batch, h, w_, p.splits, p.sps,
                      (const uint8_t*)nullptr, (int64_t)0, (const float*)nullptr, (int64_t)0, 0, 0,
                      NormTail{}, DgradParts{});
        else
            FH_LAUNCH((conv_c1_wgrad_mfma_kernel<64, false>), grid, dim3(256), 0, st, x, x_cs, dy,
                      dy_cs, part, bpart, counts, batch, h, w_, p.splits, p.sps,
                      (const uint8_t*)nullptr, (int64_t)0, (const float*)nullptr, (int64_t)0, 0, 0,
                      NormTail{}, DgradParts{});
        FH_LAUNCH_CHECK("conv2d_wgrad c1 mfma");
        if (defer_splits) {
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)part, dw, dw_cs, p.splits, cout * 9,
                                      (const float*)bpart, db, db_cs, cout, nclients, st))
            return _r;
        FH_LAUNCH_CHECK("conv2d_wgrad c1 reduce");
        return FH_OK;
    }
    if (!in_scale && conv_c1_supported(cin, cout, kh, kw, stride, pad)) {
        DWPlan p{1, 1, 1, 1, conv_c1_chunks(batch, h, w_), 1};
        const size_t need = dwgrad_ws_bytes(p, nclients, cout, 9);
        FH_REQUIRE(workspace && ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes,
                   need);
        float* part = (float*)workspace;
        const size_t wbytes = ((size_t)nclients * p.splits * cout * 9 * sizeof(float) + 255) / 256 * 256;
        float* bpart = db ? (float*)((char*)workspace + wbytes) : nullptr;
        hipStream_t st = as_stream(stream);
        FH_LAUNCH(conv_c1_wgrad_kernel<false>,
                  dim3((unsigned)p.splits, (unsigned)(cout / 8), nclients), dim3(256), 0, st, x,
                  x_cs, dy, dy_cs, part, bpart, counts, batch, h, w_, cout, p.splits,
                  (const uint8_t*)nullptr, (int64_t)0, (const float*)nullptr, (int64_t)0, 0, 0);
        FH_LAUNCH_CHECK("conv2d_wgrad c1");
        const int MN = cout * 9;
        if (defer_splits) {
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)part, dw, dw_cs, p.splits, MN, (const float*)bpart, db, db_cs, cout, nclients, st)) return _r;
        FH_LAUNCH_CHECK("conv2d_wgrad c1 reduce");
        return FH_OK;
    }
    if (aligned && dwgrad_small_supported(cin, cout, h, w_, kh, kw, stride, pad)) {
        const DWPlan p = plan_dwgrad_small(cout, batch, w_, nclients);
        const size_t need = dwgrad_ws_bytes(p, nclients, a.M, a.N);
        FH_REQUIRE(ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes, need);
        DWArgs d{};
        d.x = x; d.dy = dy; d.x_cs = x_cs; d.dy_cs = dy_cs; d.counts = counts;
        d.batch = batch; d.cin = cin; d.M = cout; d.N = a.N;
        d.splits = p.splits; d.stages_per_split = p.sps;
        d.part = (float*)workspace;
        const size_t wbytes = ((size_t)nclients * p.splits * a.M * a.N * sizeof(float) + 255) / 256 * 256;
        d.bias_part = db ? (float*)((char*)workspace + wbytes) : nullptr;
        hipStream_t st = as_stream(stream);
        dim3 grid((unsigned)p.splits, (unsigned)(cout / 32), (unsigned)nclients);
        if (w_ == 32) FH_LAUNCH((dconv_wgrad_small_kernel<32, 3>), grid, dim3(256), 0, st, d);
        else if (w_ == 16) FH_LAUNCH((dconv_wgrad_small_kernel<16, 3>), grid, dim3(256), 0, st, d);
        else FH_LAUNCH((dconv_wgrad_small_kernel<8, 3>), grid, dim3(256), 0, st, d);
        FH_LAUNCH_CHECK("conv2d_wgrad small-cin");
        const int MN = a.M * a.N;
        if (defer_splits) {
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)workspace, dw, dw_cs, p.splits, MN, (const float*)d.bias_part, db, db_cs, a.M, nclients, st)) return _r;
        FH_LAUNCH_CHECK("conv2d_wgrad reduce");
        return FH_OK;
    }
    if (aligned && dwgrad_supported(cin, cout, h, w_, kh, kw, stride, pad)) {
        const DWPlan p = plan_dwq(cout, cin, batch, w_, nclients);
        DWArgs d{};
        d.x = x; d.dy = dy; d.x_cs = x_cs; d.dy_cs = dy_cs; d.counts = counts;
        d.batch = batch; d.cin = cin; d.M = cout; d.N = a.N;
        d.splits = p.splits; d.stages_per_split = p.sps;
        d.in_scale = in_scale; d.in_shift = in_shift; d.aff_cs = aff_cs;
        hipStream_t st = as_stream(stream);
        dim3 grid((unsigned)p.splits, (unsigned)((cout / 32) * (cin / 32)), (unsigned)nclients);
        if (p.splits == 1) {  // one split per tile: dW / db straight from the kernel
            d.dw = dw; d.dw_cs = dw_cs; d.db = db; d.db_cs = db_cs;
        } else {
            const size_t need = dwgrad_ws_bytes(p, nclients, a.M, a.N);
            FH_REQUIRE(ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes, need);
            d.part = (float*)workspace;
            const size_t wbytes = ((size_t)nclients * p.splits * a.M * a.N * sizeof(float) + 255) / 256 * 256;
            d.bias_part = db ? (float*)((char*)workspace + wbytes) : nullptr;
        }
        if (p.sr * w_ == 64) {
            if (w_ == 32) FH_LAUNCH((dwgrad_q_kernel<32, 64, true>), grid, dim3(256), 0, st, d);
            else if (w_ == 16) FH_LAUNCH((dwgrad_q_kernel<16, 64, true>), grid, dim3(256), 0, st, d);
            else FH_LAUNCH((dwgrad_q_kernel<8, 64, true>), grid, dim3(256), 0, st, d);
        } else if (pair && (p.splits == 1 || defer_splits)) {  // held for the next DGRAD
            if (const int fr = flush_pending_wgrad()) return fr;
            g_pend.w = w_;
            g_pend.mode = pair;
            g_pend.grid = grid;
            g_pend.d = d;
            g_pend.st = st;
            g_pend.on = true;
            g_pend.pdy = pdy_hold;
            if (pdy_hold) g_pend.d.pdy = g_pdy.p;
        } else {
            if (w_ == 32) FH_LAUNCH((dwgrad_q_kernel<32, 128, false>), grid, dim3(256), 0, st, d);
            else if (w_ == 16) FH_LAUNCH((dwgrad_q_kernel<16, 128, false>), grid, dim3(256), 0, st, d);
            else FH_LAUNCH((dwgrad_q_kernel<8, 128, false>), grid, dim3(256), 0, st, d);
        }
        FH_LAUNCH_CHECK("conv2d_wgrad direct (quadrant waves)");
        if (p.splits == 1) return FH_OK;
        const int MN = a.M * a.N;
        if (defer_splits) {
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)workspace, dw, dw_cs, p.splits, MN, (const float*)d.bias_part, db, db_cs, a.M, nclients, st)) return _r;
        FH_LAUNCH_CHECK("conv2d_wgrad reduce");
        return FH_OK;
    }
    if (aligned && !in_scale && dwgrad_s2_supported(cin, cout, h, w_, kh, kw, stride, pad)) {
        const DWPlan p = plan_dwgrad_s2(cout, cin, batch, ow, nclients);
        const size_t need = dwgrad_ws_bytes(p, nclients, a.M, a.N);
        FH_REQUIRE(ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes, need);
        DWArgs d{};
        d.x = x; d.dy = dy; d.x_cs = x_cs; d.dy_cs = dy_cs; d.counts = counts;
        d.batch = batch; d.cin = cin; d.M = cout; d.N = a.N;
        d.splits = p.splits; d.stages_per_split = p.sps;
        d.part = (float*)workspace;
        const size_t wbytes = ((size_t)nclients * p.splits * a.M * a.N * sizeof(float) + 255) / 256 * 256;
        d.bias_part = db ? (float*)((char*)workspace + wbytes) : nullptr;
        hipStream_t st = as_stream(stream);
        dim3 grid((unsigned)p.splits, (unsigned)((cout / 64) * (cin / 32)), (unsigned)nclients);
        if (ow == 16) FH_LAUNCH((dconv_wgrad_kernel<16, 2, 1, 2, 4, 2>), grid, dim3(256), 0, st, d);
        else FH_LAUNCH((dconv_wgrad_kernel<8, 2, 1, 2, 8, 2>), grid, dim3(256), 0, st, d);
        FH_LAUNCH_CHECK("conv2d_wgrad direct s2");
        const int MN = a.M * a.N;
        if (defer_splits) {
            *defer_splits = p.splits;
            *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
            return FH_OK;
        }
        if (const int _r = splitk_sum((const float*)workspace, dw, dw_cs, p.splits, MN, (const float*)d.bias_part, db, db_cs, a.M, nclients, st)) return _r;
        FH_LAUNCH_CHECK("conv2d_wgrad s2 reduce");
        return FH_OK;
    }
    Plan p = plan_wgrad(a.M, a.N, a.K, nclients);
    const size_t need = wgrad_ws_bytes(p, nclients);
    FH_REQUIRE(ws_bytes >= need, "conv2d_wgrad: workspace %zu < %zu", ws_bytes, need);
    a.splits = p.splits;
    a.kchunk = p.kchunk;
    hipStream_t st = as_stream(stream);
    if (p.splits == 1) {  // one K pass per tile: the kernel writes dW / db directly
        a.out = dw;
        a.out_cs = dw_cs;
        a.bias_part = db;
        a.b_cs = db_cs;
        dim3 grid((unsigned)ceil_div(a.N, p.t.bn), (unsigned)ceil_div(a.M, p.t.bm),
                  (unsigned)nclients);
        rc = launch_shape<OP_WGRAD>(kh, kw, stride, p.t, grid, a, st);
        if (rc) return rc;
        FH_LAUNCH_CHECK("conv2d_wgrad");
        return FH_OK;
    }
    a.out = (float*)workspace;
    const size_t wbytes = ((size_t)nclients * p.splits * a.M * a.N * sizeof(float) + 255) / 256 * 256;
    a.bias_part = db ? (float*)((char*)workspace + wbytes) : nullptr;
    dim3 grid((unsigned)ceil_div(a.N, p.t.bn), (unsigned)ceil_div(a.M, p.t.bm),
              (unsigned)(nclients * p.splits));
    rc = launch_shape<OP_WGRAD>(kh, kw, stride, p.t, grid, a, st);
    if (rc) return rc;
    FH_LAUNCH_CHECK("conv2d_wgrad");
    const int MN = a.M * a.N;
    if (defer_splits) {
        *defer_splits = p.splits;
        *defer_boff = wslab_bias_off(nclients, p.splits, cout * cin * kh * kw);
        return FH_OK;
    }
    if (const int _r = splitk_sum((const float*)workspace, dw, dw_cs, p.splits, MN, (const float*)a.bias_part, db, db_cs, a.M, nclients, st)) return _r;
    FH_LAUNCH_CHECK("conv2d_wgrad reduce");
    return FH_OK;
}

extern "C" int fh_conv2d_wgrad(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                               float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* workspace,
                               size_t ws_bytes, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t cin, int32_t h, int32_t w_, int32_t cout,
                               int32_t kh, int32_t kw, int32_t stride, int32_t pad, void* stream) {
    return conv2d_wgrad_impl(x, x_cs, nullptr, nullptr, 0, dy, dy_cs, dw, dw_cs, db, db_cs,
                             workspace, ws_bytes, counts, nclients, batch, cin, h, w_, cout, kh,
                             kw, stride, pad, stream);
}

extern "C" int fh_conv2d_wgrad_deferred(
    const float* x, int64_t x_cs, const float* in_scale, const float* in_shift, int64_t aff_cs,
    const float* dy, int64_t dy_cs, float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* slab,
    size_t slab_bytes, const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin,
    int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad,
    int32_t* splits_out, int64_t* bias_off_out, void* stream) {
    FH_REQUIRE(splits_out && bias_off_out, "conv2d_wgrad_deferred: null output");
    FH_REQUIRE((in_scale == nullptr) == (in_shift == nullptr),
               "conv2d_wgrad_deferred: scale/shift pair");
    return conv2d_wgrad_impl(x, x_cs, in_scale, in_shift, aff_cs, dy, dy_cs, dw, dw_cs, db, db_cs,
                             slab, slab_bytes, counts, nclients, batch, cin, h, w_, cout, kh, kw,
                             stride, pad, stream, splits_out, bias_off_out);
}

extern "C" int fh_conv2d_wgrad_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                                      const float* in_shift, int64_t aff_cs, const float* dy,
                                      int64_t dy_cs, float* dw, int64_t dw_cs, float* db,
                                      int64_t db_cs, void* workspace, size_t ws_bytes,
                                      const int32_t* counts, int32_t nclients, int32_t batch,
                                      int32_t cin, int32_t h, int32_t w_, int32_t cout, int32_t kh,
                                      int32_t kw, int32_t stride, int32_t pad, void* stream) {
    FH_REQUIRE(in_scale && in_shift, "conv2d_wgrad_bnrelu: null scale/shift");
    return conv2d_wgrad_impl(x, x_cs, in_scale, in_shift, aff_cs, dy, dy_cs, dw, dw_cs, db, db_cs,
                             workspace, ws_bytes, counts, nclients, batch, cin, h, w_, cout, kh,
                             kw, stride, pad, stream);
}

// ---- linear layers: a 1x1 convolution over a 1x1 image -------------------
// Skinny DGRAD (batch <= 32 images per client, the classifier of every reference CNN): a
// weight stream, so one workgroup owns 32 input features and runs the 32 images as the
// MFMA's other dimension, the out_f reduction split over its four waves and combined
// through LDS in wave order; W arrives as 128-B rows, dY as float4 runs.  fc1 dgrad at 32
// clients: 44 us vs 81 for the implicit GEMM, fc2 12 vs 27 (tools/fc_bench.py).  FWD: see
// linear_fwd_skinny_kernel below (round 3; round 1's attempt at it lost to the implicit GEMM).
namespace fh {
constexpr int kLinearSkinny = 1;
constexpr int kSkinny32 = 1;  // skinny WGRAD / fused backward for in_f % 32 (not only % 128)

__device__ __forceinline__ float f4at(const float4& v, int q) {
    return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
}

// dX[z][b][k] = sum_m dY[z][b][m] W[z][m][k] for b < cnt; M % 32 == 0, K % (32 * KT) == 0.
// KT 32-feature tiles per workgroup: each W row is read as KT consecutive 128-B pieces
// (one DRAM page run) and every wave carries KT independent accumulator chains.
// Epilogue (fused linear backward): the gradient of the layer's input through the Dropout
// and ReLU in front of it, g = dX * keep(mask) / (1 - p) if the input (relu_ref) > 0, else 0
// (dropout_bwd_kernel's operations).
struct SkinnyBwdEpi {
    const uint8_t* mask;   // dropout keep-mask [z][b][K] (nullable)
    int64_t m_cs;
    float scale;           // 1 / (1 - p)
    const float* relu_ref; // the layer input [z][b][K]: zero where it is not > 0 (nullable)
    int64_t r_cs;
    // nullable: the layer input is a flattened 2x2 max-pool output [C][OH][OW] (SimpleCNN
    // fc1 after pool2).  dX is then written as the pool INPUT's gradient — planes xh x xw,
    // the 2OH x 2OW map in the top-left — routed to the window argmax pidx (dense
    // [C][OH][OW]) and zero elsewhere, maxpool2_bwd_kernel's values exactly (relu_ref = the
    // pooled ReLU output: the mask at the argmax)
    const uint8_t* pidx;
    int64_t pi_cs;
    int pow_, pohw, xh, xw;
};

template <int KT>
__device__ __forceinline__ void linear_dgrad_skinny_body(
        const float* __restrict__ dY, int64_t dy_cs, const float* __restrict__ W, int64_t w_cs,
        float* __restrict__ dX, int64_t dx_cs, const int32_t* __restrict__ counts, int batch,
        int K, int M, int z, int kblock, float* red, const SkinnyBwdEpi& ep) {
    const int k0 = kblock * 32 * KT;
    const int cnt = counts ? counts[z] : batch;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int r32 = lane & 31, h = lane >> 5;
    const bool yok = r32 < cnt;
    const float* yrow = dY + z * dy_cs + (int64_t)(yok ? r32 : 0) * M;   // A: image rows of dY
    const float* wcol = W + z * w_cs + k0 + r32;                          // B: W[m][k0 + lane]
    const int mw = M >> 2, mbeg = wid * mw;
    f32x16 acc[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    // software-pipelined: the next 8-m block's loads are issued before this block's MFMAs, and
    // no load sits under a branch (yrow / wcol are always in bounds; rows past the count are
    // zeroed by a select) — r05: the conditional dY load put each block's loads in a basic
    // block of their own, one dependent round trip per block
    auto ld = [&](int mb, float4& a, float (&b)[4][KT]) {
        a = *reinterpret_cast<const float4*>(yrow + mb + 4 * h);
        if (!yok) a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int t = 0; t < KT; ++t) b[q][t] = wcol[(int64_t)(mb + 4 * h + q) * K + 32 * t];
    };
    // r06: a ring of PD 8-m blocks in flight (was two): a block's 16 MFMAs (~0.4 us) hide a
    // fraction of one memory round trip, so with one block of lookahead every block waited out
    // most of a latency (KT fc1 at 8 clients, fill 0.5: 16 blocks per wave, 24.2 -> 22.4 us per
    // launch; 23 clients 47.2 -> 43.9, tools/fcab.sh, profiles/r06_fc/).  Same MFMA order.
    // (KT = 1, SimpleCNN fc1: 4 blocks per wave, +2-6 % per launch with PD = 4: kept at 2)
    constexpr int PD = KT == 4 ? 4 : 2;
    const int nb = mw / 8;
    float4 a[PD];
    float b[PD][4][KT];
#pragma unroll
    for (int i = 0; i < PD; ++i)
        if (i < nb) ld(mbeg + 8 * i, a[i], b[i]);
    for (int j0 = 0; j0 < nb; j0 += PD) {
#pragma unroll
        for (int i = 0; i < PD; ++i) {
            if (j0 + i < nb) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int t = 0; t < KT; ++t)
                        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(a[i], q), b[i][q][t],
                                                                      acc[t], 0, 0, 0);
                if (j0 + i + PD < nb) ld(mbeg + 8 * (j0 + i + PD), a[i], b[i]);
            }
        }
    }
    // waves 1..3 hand their partials to wave 0 one at a time through one wave's worth of
    // LDS (16 KB at KT = 4, so LDS does not cap the workgroups per CU); wave 0 adds them in
    // wave order
    for (int w = 1; w < 4; ++w) {
        if (wid == w) {
#pragma unroll
            for (int t = 0; t < KT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) red[(t * 16 + r) * 64 + lane] = acc[t][r];
        }
        __syncthreads();
        if (wid == 0) {
#pragma unroll
            for (int t = 0; t < KT; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[t][r] = acc[t][r] + red[(t * 16 + r) * 64 + lane];
        }
        __syncthreads();
    }
    if (wid != 0) return;
    // the epilogue's operands (keep-mask, ReLU reference, pool argmax) loaded for every element
    // first: interleaved with the dX stores (which may alias them) each element cost one
    // dependent round trip — r05: fc2's backward took ~21 us at every client count
    // r05: per 32-feature tile, the three operand streams are loaded unconditionally (a null
    // operand reads this client's dX rows instead and is discarded by a uniform select), then
    // combined — one round trip per tile (the combined form had put each load and its use in a
    // branch of its own: a dependent round trip per element and operand, 48 per tile)
    const uint8_t* dxb = reinterpret_cast<const uint8_t*>(dX + z * dx_cs);
    const uint8_t* mkp = ep.mask ? ep.mask + z * ep.m_cs : dxb;
    const float* rrp = ep.relu_ref ? ep.relu_ref + z * ep.r_cs : dX + z * dx_cs;
    const uint8_t* pap = ep.pidx ? ep.pidx + z * ep.pi_cs : dxb;
    uint32_t kp[KT][16];  // keep | relu-ok << 1 | argmax << 2
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        uint32_t mk[16], pa[16];
        float rr[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int img = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int64_t e = (int64_t)(img < cnt ? img : 0) * K + k0 + 32 * t + r32;
            mk[r] = mkp[e];
            rr[r] = rrp[e];
            pa[r] = pap[e];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
            kp[t][r] = (ep.mask ? (mk[r] ? 1u : 0u) : 1u) |
                       (ep.relu_ref ? (rr[r] > 0.f ? 2u : 0u) : 2u) | (ep.pidx ? pa[r] << 2 : 0u);
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int img = (r & 3) + 8 * (r >> 2) + 4 * h;
            if (img >= cnt) continue;
            float v = acc[t][r];
            const int64_t e = (int64_t)img * K + k0 + 32 * t + r32;
            if (ep.mask) v = (kp[t][r] & 1u) ? v * ep.scale : 0.f;
            if (ep.relu_ref && !(kp[t][r] & 2u)) v = 0.f;
            if (ep.pidx) {
                const int f = k0 + 32 * t + r32, c = f / ep.pohw, rem = f - c * ep.pohw;
                const int oh = rem / ep.pow_, ow = rem - oh * ep.pow_;
                const int a = (int)(kp[t][r] >> 2);
                float* d = dX + z * dx_cs +
                           ((int64_t)(img * (K / ep.pohw) + c) * ep.xh + 2 * oh) * ep.xw + 2 * ow;
                d[0] = a == 0 ? v : 0.f;
                d[1] = a == 1 ? v : 0.f;
                d[ep.xw] = a == 2 ? v : 0.f;
                d[ep.xw + 1] = a == 3 ? v : 0.f;
            } else {
                dX[z * dx_cs + e] = v;
            }
        }
}

template <int KT>
__global__ void __launch_bounds__(256)
linear_dgrad_skinny_kernel(const float* __restrict__ dY, int64_t dy_cs, const float* __restrict__ W,
                           int64_t w_cs, float* __restrict__ dX, int64_t dx_cs,
                           const int32_t* __restrict__ counts, int batch, int K, int M,
                           SkinnyBwdEpi ep) {
    __shared__ float red[16 * 64 * KT];
    linear_dgrad_skinny_body<KT>(dY, dy_cs, W, w_cs, dX, dx_cs, counts, batch, K, M, blockIdx.y,
                                 blockIdx.x, red, ep);
}

// dW[z][m][k] = sum_{b < cnt} dY[z][b][m] X[z][b][k] (and db[z][m] = sum_b dY[z][b][m]):
// the reduction is only the images, so the layer is a write stream of dW.  One wave = one
// 32 (m) x 32 (k) tile from 16 MFMAs over the 32 image pairs; a workgroup = 32 m x 128 k.
// Bias: the k-tile-0 workgroups, one lane per m, images in order.
__device__ __forceinline__ void linear_wgrad_skinny_body(
        const float* __restrict__ X, int64_t x_cs, const float* __restrict__ dY, int64_t dy_cs,
        float* __restrict__ dW, int64_t dw_cs, float* __restrict__ db, int64_t db_cs,
        const int32_t* __restrict__ counts, int batch, int K, int M, int z, int kblock,
        int mblock, const float* __restrict__ rowscale = nullptr) {
    // rowscale (nullable, [client][batch]): dY row b scaled by rowscale[z][b] on load — the
    // fp32 products fh_scale_rows would store (DP-SGD's clipped linear-layer sums)
    const int m0 = mblock * 32;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int k0 = kblock * 128 + wid * 32;
    if (k0 >= K) return;  // K % 128 != 0 (K % 32 == 0): the last block's spare waves
    const int cnt = counts ? counts[z] : batch;
    const int r32 = lane & 31, h = lane >> 5;
    const bool mok = m0 + r32 < M;
    const float* yz = dY + z * dy_cs + m0 + r32;   // A[i = m][b] = dY[b][m0 + lane]
    const float* xz = X + z * x_cs + k0 + r32;     // B[b][j = k] = X[b][k0 + lane]
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // row scales: lane l holds row l's (one coalesced load), image b's comes by a lane shuffle
    const float rs_l = (rowscale && r32 < cnt) ? rowscale[(int64_t)z * batch + r32] : 1.f;
    // every image's operands loaded first, from in-bounds addresses (rows past the count and
    // columns past M read row 0 / column m0 and are zeroed by a select): r05 — the conditional
    // loads had put each image pair's loads and MFMA in a basic block of their own, 16
    // dependent round trips per tile
    const float* yzc = dY + z * dy_cs + (mok ? m0 + r32 : 0);
    float av[16], bv[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        const int b = 2 * p + h, bc = b < cnt ? b : 0;
        av[p] = yzc[(int64_t)bc * M];
        bv[p] = xz[(int64_t)bc * K];
    }
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        const int b = 2 * p + h;
        const bool ok = b < cnt;
        float a = ok && mok ? av[p] : 0.f;
        const float rsb = __shfl(rs_l, b, 64);
        if (rowscale && ok) a = rsb * a;
        const float bb = ok ? bv[p] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
    }
    float* wz = dW + z * dw_cs + k0 + r32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) wz[(int64_t)m * K] = acc[r];
    }
    if (db && kblock == 0 && wid == 0 && h == 0 && mok) {
        // every image's term loaded first, then added in image order (the loop's loads had
        // waited for each other: 32 dependent round trips in the kernel's tail — r04)
        // (r05: from in-bounds addresses, selects after — the conditional loads had sat in
        // branches with their uses under a row scale)
        const float* rsz = rowscale ? rowscale + (int64_t)z * batch : yz;
        float t[32], sc[32];
#pragma unroll
        for (int b = 0; b < 32; ++b) {
            const int bc = b < cnt ? b : 0;
            t[b] = yz[(int64_t)bc * M];
            sc[b] = rsz[rowscale ? bc : 0];
        }
#pragma unroll
        for (int b = 0; b < 32; ++b) t[b] = b < cnt ? (rowscale ? sc[b] * t[b] : t[b]) : 0.f;
        float v = 0.f;
#pragma unroll
        for (int b = 0; b < 32; ++b)
            if (b < cnt) v += t[b];
        db[z * db_cs + m0 + r32] = v;
    }
}

__global__ void __launch_bounds__(256)
linear_wgrad_skinny_kernel(const float* __restrict__ X, int64_t x_cs, const float* __restrict__ dY,
                           int64_t dy_cs, float* __restrict__ dW, int64_t dw_cs,
                           float* __restrict__ db, int64_t db_cs,
                           const int32_t* __restrict__ counts, int batch, int K, int M,
                           const float* __restrict__ rowscale = nullptr) {
    // XCD-aware order: workgroups b and b + 8 share an XCD (round-robin dispatch), so the
    // logical workgroup L = (b % 8) * (N / 8) + b / 8 puts each client's tiles — which all
    // read that client's X and dY — on one XCD's L2 instead of all eight
    const int gx = gridDim.x, gy = gridDim.y;
    const int N = gx * gy * gridDim.z;
    int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if ((N & 7) == 0) b = (b & 7) * (N >> 3) + (b >> 3);
    const int kb = b % gx, rest = b / gx;
    linear_wgrad_skinny_body(X, x_cs, dY, dy_cs, dW, dw_cs, db, db_cs, counts, batch, K, M,
                             rest / gy, kb, rest % gy, rowscale);
}

// Several linear layers' weight gradients in one launch (r05, DP-SGD's pass 2: fc2's and
// fc1's clipped sums on the same row scales were two dependent launches): the grid is the
// layers' skinny-WGRAD grids one after another, each block running linear_wgrad_skinny_body
// for its layer with that layer's own XCD-aware order — the same tiles, the same bits.
struct LinWgLayer {
    const float* x;
    int64_t x_cs;
    const float* dy;
    int64_t dy_cs;
    float* dw;
    int64_t dw_cs;
    float* db;
    int64_t db_cs;
    int K, M, gx, gy, nblk;  // in_f, out_f, grid x / y, blocks (gx * gy * clients)
};
constexpr int kMaxLinWg = 4;
struct LinWgSet {
    LinWgLayer l[kMaxLinWg];
    int n;
};

__global__ void __launch_bounds__(256)
linear_wgrad_skinny_multi_kernel(const LinWgSet set, const int32_t* __restrict__ counts, int batch,
                                 const float* __restrict__ rowscale) {
    int b = blockIdx.x, li = 0;
    while (li + 1 < set.n && b >= set.l[li].nblk) {
        b -= set.l[li].nblk;
        ++li;
    }
    const LinWgLayer& L = set.l[li];
    const int N = L.nblk;
    if ((N & 7) == 0) b = (b & 7) * (N >> 3) + (b >> 3);  // as linear_wgrad_skinny_kernel
    const int kb = b % L.gx, rest = b / L.gx;
    linear_wgrad_skinny_body(L.x, L.x_cs, L.dy, L.dy_cs, L.dw, L.dw_cs, L.db, L.db_cs, counts,
                             batch, L.K, L.M, rest / L.gy, kb, rest % L.gy, rowscale);
}

// A whole linear backward in one launch: workgroups [0, nw) of each client are the skinny
// WGRAD tiles (in_f/128 x ceil(out_f/32)), the rest the skinny DGRAD tiles with the Dropout /
// ReLU backward of the layer's input fused into the epilogue — three launches (wgrad, dgrad,
// dropout_bwd) become one.  grid = (nw + nd, clients).
template <int KT>
__global__ void __launch_bounds__(256)
linear_bwd_fused_kernel(const float* __restrict__ X, int64_t x_cs, const float* __restrict__ dY,
                        int64_t dy_cs, const float* __restrict__ W, int64_t w_cs,
                        float* __restrict__ dW, int64_t dw_cs, float* __restrict__ db,
                        int64_t db_cs, float* __restrict__ dX, int64_t dx_cs, SkinnyBwdEpi ep,
                        const int32_t* __restrict__ counts, int batch, int K, int M, int nw) {
    __shared__ float red[16 * 64 * KT];
    const int z = blockIdx.y, bx = blockIdx.x;
    if (bx < nw) {
        const int kt = (K + 127) / 128;
        linear_wgrad_skinny_body(X, x_cs, dY, dy_cs, dW, dw_cs, db, db_cs, counts, batch, K, M,
                                 z, bx % kt, bx / kt);
    } else {
        linear_dgrad_skinny_body<KT>(dY, dy_cs, W, w_cs, dX, dx_cs, counts, batch, K, M, z,
                                     bx - nw, red, ep);
    }
}

static bool skinny_aligned(const void* p, int64_t cs) {
    return ((uintptr_t)p % 16 == 0) && cs % 4 == 0;
}

// Skinny linear FORWARD (batch <= 32 images per client, in_f % 32 == 0: SimpleCNN fc1
// 3136->128, CIFAR10CNN fc1 2048->512 / fc2 512->256): y[img][o] = sum_k x[img][k] w[o][k]
// (+ bias, ReLU, dropout).  A stream of W — each weight feeds at most 32 images — so the
// operands go from global memory straight to registers, no LDS staging: per 32-k block a lane
// loads 64 contiguous bytes of one x row (img = lane & 31) and one w row (o = lane & 31), two
// lanes per 128-B line, and the block's 16 v_mfma_f32_32x32x2_f32 pair k = (k0 + 4q + j,
// k0 + 16 + 4q + j) on the two lane halves.  A wave owns 32 outputs x all 32 images (one
// accumulator); a workgroup = OT such output tiles x KG = 4 / OT k-groups over one k-chunk
// (the k-groups take interleaved blocks, so the four waves read neighbouring pieces of the
// same rows, and are combined through LDS in k-group order).  D blocks of loads stay in
// flight ahead of the MFMAs (round 1's skinny FWD ran one dependent chain over all of K per
// wave with nothing in flight: 123 vs 57 us).  The workgroups of one client sit on one XCD
// (x read once per L2).  splits == 1: bias / ReLU / dropout in the epilogue; else a
// [client][split][32][out_f] slab, summed in split order by linear_fwd_epilogue_kernel.
template <int D, int OT>
__global__ void __launch_bounds__(256)
linear_fwd_skinny_kernel(const float* __restrict__ X, int64_t x_cs, const float* __restrict__ W,
                         int64_t w_cs, const float* __restrict__ bias, int64_t b_cs,
                         float* __restrict__ Y, int64_t y_cs, float* __restrict__ part,
                         const int32_t* __restrict__ counts, int batch, int K, int M, int kbps,
                         int relu, DropArgs drop) {
    constexpr int KG = 4 / OT;
    __shared__ float red[KG > 1 ? (KG - 1) * OT * 16 * 64 : 1];
    const int gx = gridDim.x, gy = gridDim.y;  // x: splits, y: output groups, z: clients
    const int N = gx * gy * gridDim.z;
    int b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if ((N & 7) == 0) b = (b & 7) * (N >> 3) + (b >> 3);  // XCD-aware, see wgrad_skinny
    const int s = b % gx, rest = b / gx, og = rest % gy, z = rest / gy;
    const int cnt = counts ? counts[z] : batch;
    if (cnt <= 0) return;  // workgroup-uniform
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int ot = wid % OT, kg = wid / OT;
    const int r = lane & 31, h = lane >> 5;
    const int o0 = (og * OT + ot) * 32;
    const bool active = o0 < M;  // wave-uniform; inactive waves still meet the barrier
    const int kb0 = s * kbps;
    const int nkb = min(kbps, K / 32 - kb0);
    const int nmine = nkb > kg ? (nkb - kg + KG - 1) / KG : 0;  // blocks kg, kg + KG, ...
    // rows past the batch / the outputs read a valid row and are never stored: an A row
    // only reaches its own D row, a B column only its own D column
    const float* xk = X + z * x_cs + (int64_t)min(r, cnt - 1) * K + (int64_t)(kb0 + kg) * 32 + 16 * h;
    const float* wk = W + z * w_cs + (int64_t)min(o0 + r, M - 1) * K + (int64_t)(kb0 + kg) * 32 + 16 * h;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (active) {
        float4 xa[D][4], wa[D][4];
#pragma unroll
        for (int d = 0; d < D; ++d)
            if (d < nmine) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xa[d][q] = *reinterpret_cast<const float4*>(xk + d * KG * 32 + 4 * q);
                    wa[d][q] = *reinterpret_cast<const float4*>(wk + d * KG * 32 + 4 * q);
                }
            }
        for (int b0 = 0; b0 < nmine; b0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int bb = b0 + d;
                if (bb < nmine) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[d][q].x, wa[d][q].x, acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[d][q].y, wa[d][q].y, acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[d][q].z, wa[d][q].z, acc, 0, 0, 0);
                        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[d][q].w, wa[d][q].w, acc, 0, 0, 0);
                    }
                    if (bb + D < nmine) {
                        const int64_t off = (int64_t)(bb + D) * KG * 32;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            xa[d][q] = *reinterpret_cast<const float4*>(xk + off + 4 * q);
                            wa[d][q] = *reinterpret_cast<const float4*>(wk + off + 4 * q);
                        }
                    }
                }
            }
        }
    }
    if constexpr (KG > 1) {  // k-groups 1.. hand their sums to k-group 0, added in order
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) red[(((kg - 1) * OT + ot) * 16 + i) * 64 + lane] = acc[i];
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KG; ++g)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[i] += red[(((g - 1) * OT + ot) * 16 + i) * 64 + lane];
    }
    const int o = o0 + r;
    if (!active || o >= M) return;
    if (gx == 1) {
        const float bv = bias ? bias[z * b_cs + o] : 0.f;
        const DropKey dk = drop_key(drop, z);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int img = (i & 3) + 8 * (i >> 2) + 4 * h;
            if (img < cnt) {
                float v = acc[i];
                if (bias) v = v + bv;
                if (relu) v = fmaxf(v, 0.f);
                const int64_t e = (int64_t)img * M + o;
                if (drop.mode) v = apply_dropout(drop, dk, z, e, v);
                Y[z * y_cs + e] = v;
            }
        }
    } else {
        float* pp = part + ((int64_t)z * gx + s) * 32 * M + o;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int img = (i & 3) + 8 * (i >> 2) + 4 * h;
            if (img < cnt) pp[(int64_t)img * M] = acc[i];
        }
    }
}

// linear_fwd_skinny's split reduction: y[z][e] = epilogue(sum_s part[z][s][e]), e = img*M + o
// (splitk_epilogue_kernel's operations and order: slabs in split order, + bias, ReLU, dropout)
__global__ void __launch_bounds__(256)
linear_fwd_epilogue_kernel(const float* __restrict__ part, int splits, int M,
                           float* __restrict__ Y, int64_t y_cs, const float* __restrict__ bias,
                           int64_t b_cs, int relu, const int32_t* __restrict__ counts, int batch,
                           DropArgs drop) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= cnt * M) return;
    const float* p = part + (int64_t)z * splits * 32 * M + e;
    const int64_t ss = (int64_t)32 * M;
    float v = 0.f;
    for (int i0 = 0; i0 < splits; i0 += 8) {
        float t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = i0 + j < splits ? p[(i0 + j) * ss] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (i0 + j < splits) v += t[j];
    }
    if (bias) v = v + bias[z * b_cs + e % M];
    if (relu) v = fmaxf(v, 0.f);
    if (drop.mode) v = apply_dropout(drop, drop_key(drop, z), z, e, v);
    Y[z * y_cs + e] = v;
}

// Split plan of linear_fwd_skinny: enough k-chunks that (output groups x clients x chunks)
// reaches fill(kLfTarget) workgroups, each k-group of a chunk >= kLfMinKb 32-k blocks
// (r03 sweeps, profiles/r03_lf/: target 512, 4 blocks, two blocks of loads in flight, one
// output tile per workgroup)
constexpr int kLfTarget = 512;
constexpr int kLfMinKb = 4;
// 32-k blocks of loads in flight per wave (r03: 2; r06 measured 4: within noise at C = 1 / 8,
// +1-3 % per launch at 21-23 clients, tools/fcab.sh — kept at 2)
constexpr int kLfDepth = 2;

static bool linear_fwd_skinny_ok(int batch, int in_f, int out_f) {
    return kLinearSkinny && kLinearSkinny != 3 && batch > 0 && batch <= 32 && in_f > 0 &&
           in_f % 32 == 0 && out_f > 0;
}

static void plan_lin_fwd(int nclients, int in_f, int out_f, int64_t target, int& splits,
                         int& kbps) {
    const int kb = in_f / 32;
    const int64_t tiles = (int64_t)ceil_div(out_f, 32) * std::max(nclients, 1);
    int64_t want = ceil_div(target, tiles);
    want = std::min<int64_t>(want, std::max(1, kb / (kLfMinKb * 4)));
    want = std::max<int64_t>(want, 1);
    kbps = (int)ceil_div(kb, want);
    splits = (int)ceil_div(kb, kbps);
}

static int linear_fwd_skinny(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                             const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                             const int32_t* counts, int nclients, int batch, int in_f, int out_f,
                             int relu, const DropArgs& drop, void* workspace, size_t ws_bytes,
                             hipStream_t st) {
    int splits, kbps;
    plan_lin_fwd(nclients, in_f, out_f, fill(kLfTarget), splits, kbps);
    const dim3 grid((unsigned)splits, (unsigned)ceil_div(out_f, 32), (unsigned)nclients);
    float* part = nullptr;
    if (splits > 1) {
        const size_t need = (size_t)nclients * splits * 32 * out_f * sizeof(float);
        FH_REQUIRE(workspace && ws_bytes >= need, "linear_fwd: workspace %zu < %zu", ws_bytes, need);
        part = (float*)workspace;
    }
    FH_LAUNCH((linear_fwd_skinny_kernel<kLfDepth, 1>), grid, dim3(256), 0, st, x, x_cs, w, w_cs, bias,
              b_cs, y, y_cs, part, counts, batch, in_f, out_f, kbps, relu, drop);
    if (splits > 1)
        FH_LAUNCH(linear_fwd_epilogue_kernel, dim3((unsigned)ceil_div(32 * out_f, 256), nclients),
                  dim3(256), 0, st, (const float*)part, splits, out_f, y, y_cs, bias, b_cs, relu,
                  counts, batch, drop);
    return FH_OK;
}
}  // namespace fh

extern "C" size_t fh_linear_fwd_workspace(int32_t nclients, int32_t batch, int32_t in_f,
                                          int32_t out_f) {
    size_t ws = fh_conv2d_fwd_workspace(nclients, batch, in_f, 1, 1, out_f, 1, 1, 1, 0);
    if (fh::linear_fwd_skinny_ok(batch, in_f, out_f) && nclients > 0) {
        int splits, kbps;  // the whole-chip plan has the most splits of any fill fraction
        fh::plan_lin_fwd(nclients, in_f, out_f, fh::kLfTarget, splits, kbps);
        if (splits > 1)
            ws = std::max(ws, (size_t)nclients * splits * 32 * out_f * sizeof(float));
    }
    return ws;
}

extern "C" size_t fh_linear_dgrad_workspace(int32_t nclients, int32_t batch, int32_t in_f,
                                            int32_t out_f) {
    return fh_conv2d_dgrad_workspace(nclients, batch, in_f, 1, 1, out_f, 1, 1, 1, 0);
}

extern "C" int fh_linear_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                             const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                             const int32_t* counts, int32_t nclients, int32_t batch, int32_t in_f,
                             int32_t out_f, int32_t relu, void* workspace, size_t ws_bytes,
                             void* stream) {
    if (fh::linear_fwd_skinny_ok(batch, in_f, out_f) && nclients > 0 && x && w && y &&
        fh::skinny_aligned(x, x_cs) && fh::skinny_aligned(w, w_cs))
        return fh::linear_fwd_skinny(x, x_cs, w, w_cs, bias, b_cs, y, y_cs, counts, nclients,
                                     batch, in_f, out_f, relu, fh::DropArgs{}, workspace,
                                     ws_bytes, fh::as_stream(stream));
    return fh_conv2d_fwd(x, x_cs, w, w_cs, bias, b_cs, y, y_cs, counts, nclients, batch, in_f, 1, 1,
                         out_f, 1, 1, 1, 0, relu, workspace, ws_bytes, stream);
}

// fh_linear_fwd + fh_dropout_fwd (F.dropout after the layer's ReLU) in one product: the
// dropout runs in the FWD epilogue (or the split-K epilogue), same keep-mask draws and
// element order as fh_dropout_fwd, so y equals dropout_fwd(linear_fwd(x)).
extern "C" int fh_linear_fwd_dropout(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                                     const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                                     uint8_t* mask, int64_t m_cs, const int32_t* counts,
                                     int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f,
                                     int32_t relu, int32_t drop_mode, float p_drop,
                                     uint64_t seed, const uint64_t* seed_dev, void* workspace,
                                     size_t ws_bytes, void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, in_f, 1, 1, out_f, 1, 1, 1, 0, oh, ow);
    if (rc) return rc;
    FH_REQUIRE((drop_mode == 1 || drop_mode == 2) && mask, "linear_fwd_dropout: mask mode");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "linear_fwd_dropout: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && w && y, "linear_fwd_dropout: null pointer");
    ConvArgs a = make_args(batch, in_f, 1, 1, out_f, 1, 1, 0, counts);
    a.x = x; a.wt = w; a.bias = bias; a.out = y;
    a.x_cs = x_cs; a.w_cs = w_cs; a.b_cs = b_cs; a.out_cs = y_cs;
    a.relu = relu;
    a.M = out_f; a.N = batch; a.K = in_f;
    const float keep = 1.0f - p_drop;
    a.drop = DropArgs{mask, m_cs, drop_mode, keep, 1.0f / keep, seed, seed_dev};
    if (linear_fwd_skinny_ok(batch, in_f, out_f) && skinny_aligned(x, x_cs) &&
        skinny_aligned(w, w_cs))
        return linear_fwd_skinny(x, x_cs, w, w_cs, bias, b_cs, y, y_cs, counts, nclients, batch,
                                 in_f, out_f, relu, a.drop, workspace, ws_bytes,
                                 as_stream(stream));
    return run_mn<OP_FWD>(a, 1, 1, 1, nclients, workspace, ws_bytes, y, y_cs, bias, b_cs, relu, 0,
                          1, as_stream(stream), "linear_fwd_dropout");
}

extern "C" int fh_linear_dgrad(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs,
                               float* dx, int64_t dx_cs, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t in_f, int32_t out_f, void* workspace,
                               size_t ws_bytes, void* stream) {
    if (kLinearSkinny && nclients > 0 && batch <= 32 && in_f % 32 == 0 && out_f % 32 == 0 &&
        in_f > 0 && out_f > 0 && dy && w && dx && skinny_aligned(dy, dy_cs) && w_cs % 4 == 0) {
        // four k-tiles per workgroup once that still fills the chip (fc1 at 32 clients:
        // 44 us vs 75; with few clients the one-tile form keeps more workgroups)
        if (in_f % 128 == 0 && kLinearSkinny != 2 &&
            (int64_t)(in_f / 128) * nclients >= fill(256))
            FH_LAUNCH(linear_dgrad_skinny_kernel<4>, dim3((unsigned)(in_f / 128), nclients),
                               dim3(256), 0, as_stream(stream), dy, dy_cs, w, w_cs, dx, dx_cs,
                               counts, batch, in_f, out_f, SkinnyBwdEpi{nullptr, 0, 1.f, nullptr, 0, nullptr, 0, 1, 1, 0, 0});
        else
            FH_LAUNCH(linear_dgrad_skinny_kernel<1>, dim3((unsigned)(in_f / 32), nclients),
                               dim3(256), 0, as_stream(stream), dy, dy_cs, w, w_cs, dx, dx_cs,
                               counts, batch, in_f, out_f, SkinnyBwdEpi{nullptr, 0, 1.f, nullptr, 0, nullptr, 0, 1, 1, 0, 0});
        FH_LAUNCH_CHECK("linear_dgrad skinny");
        return FH_OK;
    }
    return fh_conv2d_dgrad(dy, dy_cs, w, w_cs, dx, dx_cs, counts, nclients, batch, in_f, 1, 1,
                           out_f, 1, 1, 1, 0, 0, workspace, ws_bytes, stream);
}

// Fused linear backward (fh_linear_wgrad + fh_linear_dgrad + the Dropout/ReLU backward of
// the layer input, fh_dropout_bwd) in one launch: batch <= 32, in_f % 128 == 0,
// out_f % 32 == 0, 16-B aligned dY rows; FH_E_UNSUPPORTED otherwise (the caller then issues
// the three entry points).  mask / relu_ref nullable; db nullable.
static int linear_bwd_fused_impl(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                                 const float* w, int64_t w_cs, float* dw, int64_t dw_cs,
                                 float* db, int64_t db_cs, float* dx, int64_t dx_cs,
                                 const SkinnyBwdEpi& ep, const int32_t* counts, int32_t nclients,
                                 int32_t batch, int32_t in_f, int32_t out_f, void* stream) {
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && w && dw && dx, "linear_bwd_fused: null pointer");
    if (!(batch <= 32 && in_f % (kSkinny32 ? 32 : 128) == 0 && out_f % 32 == 0 &&
          skinny_aligned(dy, dy_cs) && w_cs % 4 == 0)) {
        set_error("linear_bwd_fused: needs batch <= 32, in_f %% 32 == 0, out_f %% 32 == 0 and "
                  "aligned dY (got %d, %d, %d)", batch, in_f, out_f);
        return FH_E_UNSUPPORTED;
    }
    const int kb = (int)ceil_div(in_f, 128);  // WGRAD k-blocks (spare waves return)
    const int nw = kb * (int)ceil_div(out_f, 32);
    if (kLinearSkinny != 2 && in_f % 128 == 0 && (int64_t)kb * nclients >= fill(256)) {
        // wide launches: the two roles as two kernels — in one grid every WGRAD workgroup
        // would carry the DGRAD role's 48 KB of LDS and stream dW at 3 workgroups per CU
        // (fc1 at 32 clients: 190 us fused vs ~105 us as two launches).  SimpleCNN's fc1
        // (in_f = 3136, one 32-feature DGRAD tile per workgroup) stays one launch at every
        // width (r04: one launch less per K2 step)
        FH_LAUNCH(linear_wgrad_skinny_kernel,
                  dim3((unsigned)kb, (unsigned)ceil_div(out_f, 32), nclients),
                  dim3(256), 0, as_stream(stream), x, x_cs, dy, dy_cs, dw, dw_cs, db, db_cs,
                  counts, batch, in_f, out_f, (const float*)nullptr);
        FH_LAUNCH_CHECK("linear_bwd_fused wgrad");
        if (in_f % 128 == 0)
            FH_LAUNCH(linear_dgrad_skinny_kernel<4>, dim3((unsigned)(in_f / 128), nclients),
                      dim3(256), 0, as_stream(stream), dy, dy_cs, w, w_cs, dx, dx_cs, counts,
                      batch, in_f, out_f, ep);
        else  // SimpleCNN fc1 (3136 = 98 x 32): one 32-feature tile per workgroup
            FH_LAUNCH(linear_dgrad_skinny_kernel<1>, dim3((unsigned)(in_f / 32), nclients),
                      dim3(256), 0, as_stream(stream), dy, dy_cs, w, w_cs, dx, dx_cs, counts,
                      batch, in_f, out_f, ep);
    } else
        FH_LAUNCH(linear_bwd_fused_kernel<1>, dim3((unsigned)(nw + in_f / 32), nclients),
                  dim3(256), 0, as_stream(stream), x, x_cs, dy, dy_cs, w, w_cs, dw, dw_cs, db,
                  db_cs, dx, dx_cs, ep, counts, batch, in_f, out_f, nw);
    FH_LAUNCH_CHECK("linear_bwd_fused");
    return FH_OK;
}

extern "C" int fh_linear_bwd_fused(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                                   const float* w, int64_t w_cs, float* dw, int64_t dw_cs,
                                   float* db, int64_t db_cs, float* dx, int64_t dx_cs,
                                   const uint8_t* mask, int64_t m_cs, float p_drop,
                                   const float* relu_ref, int64_t r_cs, const int32_t* counts,
                                   int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f,
                                   void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && in_f > 0 && out_f > 0, "linear_bwd_fused: bad shape");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "linear_bwd_fused: p=%g", p_drop);
    const SkinnyBwdEpi ep{mask, m_cs, 1.0f / (1.0f - p_drop), relu_ref, r_cs, nullptr, 0, 1, 1, 0, 0};
    return linear_bwd_fused_impl(x, x_cs, dy, dy_cs, w, w_cs, dw, dw_cs, db, db_cs, dx, dx_cs, ep,
                                 counts, nclients, batch, in_f, out_f, stream);
}

// fh_linear_bwd_fused for a layer whose input x is a flattened 2x2 max-pool output of
// ReLU'd maps [C][OH][OW] (SimpleCNN fc1 after pool2, models_pytorch.py:91-95): dX is written
// as the gradient of the POOL INPUT (fh_maxpool2_bwd's output, planes xh x xw with the
// 2OH x 2OW map in the top-left corner, other elements untouched), routed to the window
// argmax pidx (dense [C][OH][OW]) with the ReLU mask x > 0 at it — the separate
// fh_maxpool2_bwd launch and the pooled gradient tensor disappear.  Same values bit for bit.
extern "C" int fh_linear_bwd_fused_pool(const float* x, int64_t x_cs, const float* dy,
                                        int64_t dy_cs, const float* w, int64_t w_cs, float* dw,
                                        int64_t dw_cs, float* db, int64_t db_cs, float* dx,
                                        int64_t dx_cs, const uint8_t* pidx, int64_t pi_cs,
                                        const int32_t* counts, int32_t nclients, int32_t batch,
                                        int32_t C, int32_t OH, int32_t OW, int32_t xh, int32_t xw,
                                        int32_t out_f, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && OH > 0 && OW > 0 && xh >= 2 * OH &&
               xw >= 2 * OW && out_f > 0, "linear_bwd_fused_pool: bad shape");
    FH_REQUIRE(pidx || nclients == 0, "linear_bwd_fused_pool: null argmax");
    const SkinnyBwdEpi ep{nullptr, 0, 1.f, x, x_cs, pidx, pi_cs, OW, OH * OW, xh, xw};
    return linear_bwd_fused_impl(x, x_cs, dy, dy_cs, w, w_cs, dw, dw_cs, db, db_cs, dx, dx_cs, ep,
                                 counts, nclients, batch, C * OH * OW, out_f, stream);
}

extern "C" size_t fh_linear_wgrad_workspace(int32_t nclients, int32_t batch, int32_t in_f,
                                            int32_t out_f) {
    return fh_conv2d_wgrad_workspace(nclients, batch, in_f, 1, 1, out_f, 1, 1, 1, 0);
}

extern "C" int fh_linear_wgrad_rowscale(const float* x, int64_t x_cs, const float* dy,
                                        int64_t dy_cs, const float* rowscale, float* dw,
                                        int64_t dw_cs, float* db, int64_t db_cs,
                                        const int32_t* counts, int32_t nclients, int32_t batch,
                                        int32_t in_f, int32_t out_f, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && batch <= 32 && in_f > 0 && in_f % 32 == 0 &&
                   out_f > 0, "linear_wgrad_rowscale: batch <= 32 and in_f %% 32 == 0 (got %d, %d)",
               batch, in_f);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && dw && rowscale, "linear_wgrad_rowscale: null pointer");
    FH_LAUNCH(linear_wgrad_skinny_kernel,
              dim3((unsigned)ceil_div(in_f, 128), (unsigned)ceil_div(out_f, 32), nclients),
              dim3(256), 0, as_stream(stream), x, x_cs, dy, dy_cs, dw, dw_cs, db, db_cs, counts,
              batch, in_f, out_f, rowscale);
    FH_LAUNCH_CHECK("linear_wgrad_rowscale");
    return FH_OK;
}

extern "C" int fh_linear_wgrad_rowscale_multi(const fh_linear_wgrad_src* layers, int32_t nlayers,
                                              const float* rowscale, const int32_t* counts,
                                              int32_t nclients, int32_t batch, void* stream) {
    FH_REQUIRE(nlayers >= 1 && nlayers <= kMaxLinWg && layers,
               "linear_wgrad_rowscale_multi: 1..%d layers (got %d)", kMaxLinWg, nlayers);
    FH_REQUIRE(nclients >= 0 && batch > 0 && batch <= 32,
               "linear_wgrad_rowscale_multi: batch <= 32 (got %d)", batch);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(rowscale, "linear_wgrad_rowscale_multi: null row scales");
    LinWgSet set{};
    set.n = nlayers;
    int64_t total = 0;
    for (int i = 0; i < nlayers; ++i) {
        const fh_linear_wgrad_src& q = layers[i];
        FH_REQUIRE(q.x && q.dy && q.dw && q.in_f > 0 && q.in_f % 32 == 0 && q.out_f > 0,
                   "linear_wgrad_rowscale_multi: layer %d (in_f %d, out_f %d)", i, q.in_f,
                   q.out_f);
        LinWgLayer& L = set.l[i];
        L.x = q.x; L.x_cs = q.x_cs; L.dy = q.dy; L.dy_cs = q.dy_cs;
        L.dw = q.dw; L.dw_cs = q.dw_cs; L.db = q.db; L.db_cs = q.db_cs;
        L.K = q.in_f; L.M = q.out_f;
        L.gx = (int)ceil_div(q.in_f, 128);
        L.gy = (int)ceil_div(q.out_f, 32);
        const int64_t nb = (int64_t)L.gx * L.gy * nclients;
        FH_REQUIRE(nb < (1ll << 30), "linear_wgrad_rowscale_multi: grid");
        L.nblk = (int)nb;
        total += nb;
    }
    FH_REQUIRE(total < (1ll << 31), "linear_wgrad_rowscale_multi: grid");
    FH_LAUNCH(linear_wgrad_skinny_multi_kernel, dim3((unsigned)total), dim3(256), 0,
              as_stream(stream), set, counts, batch, rowscale);
    FH_LAUNCH_CHECK("linear_wgrad_rowscale_multi");
    return FH_OK;
}

extern "C" int fh_linear_wgrad(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                               float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* workspace,
                               size_t ws_bytes, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t in_f, int32_t out_f, void* stream) {
    if (kLinearSkinny && nclients > 0 && batch <= 32 && in_f % (kSkinny32 ? 32 : 128) == 0 &&
        out_f > 0 && x && dy && dw) {
        FH_LAUNCH(linear_wgrad_skinny_kernel,
                           dim3((unsigned)ceil_div(in_f, 128), (unsigned)ceil_div(out_f, 32), nclients),
                           dim3(256), 0, as_stream(stream), x, x_cs, dy, dy_cs, dw, dw_cs, db, db_cs,
                           counts, batch, in_f, out_f, (const float*)nullptr);
        FH_LAUNCH_CHECK("linear_wgrad skinny");
        return FH_OK;
    }
    return fh_conv2d_wgrad(x, x_cs, dy, dy_cs, dw, dw_cs, db, db_cs, workspace, ws_bytes, counts,
                           nclients, batch, in_f, 1, 1, out_f, 1, 1, 1, 0, stream);
}

// ---- DP-SGD: per-sample squared gradient norms of a conv layer --------------
// One WGRAD split per image (K = that image's pixels): each workgroup holds a tile
// of dW_i and reduces it to a sum of squares; conv_sq_reduce adds the tiles of each
// (client, image) in a fixed order into sqnorm[z][img] (double, accumulated over layers).
namespace fh {
__global__ void __launch_bounds__(256)
conv_sq_reduce_kernel(const float* __restrict__ part, int tiles, int batch,
                      const int32_t* __restrict__ counts, double* __restrict__ sqnorm) {
    const int z = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int cnt = counts ? counts[z] : batch;
    if (i >= batch) return;
    double s = 0.0;
    if (i < cnt) {
        const float* p = part + ((int64_t)z * batch + i) * tiles;
        for (int t = 0; t < tiles; ++t) s += (double)p[t];
    }
    sqnorm[(int64_t)z * batch + i] += s;
}
}  // namespace fh

static Plan plan_persample(int M, int N, int ohw, int batch) {
    Plan p{pick_wgrad_tile(M), batch, ohw, M, N, batch * ohw};
    return p;
}

extern "C" size_t fh_conv2d_persample_sqnorm_workspace(int32_t nclients, int32_t batch,
                                                       int32_t cin, int32_t h, int32_t w_,
                                                       int32_t cout, int32_t kh, int32_t kw,
                                                       int32_t stride, int32_t pad) {
    int oh = (h + 2 * pad - kh) / stride + 1, ow = (w_ + 2 * pad - kw) / stride + 1;
    if (oh <= 0 || ow <= 0 || nclients <= 0) return 0;
    const Plan p = plan_persample(cout, cin * kh * kw, oh * ow, batch);
    const int64_t tiles = ceil_div(p.N, p.t.bn) * ceil_div(p.M, p.t.bm);
    return (size_t)nclients * batch * tiles * sizeof(float);
}

extern "C" int fh_conv2d_persample_sqnorm(const float* x, int64_t x_cs, const float* dy,
                                          int64_t dy_cs, int32_t with_bias, double* sqnorm,
                                          void* workspace, size_t ws_bytes,
                                          const int32_t* counts, int32_t nclients, int32_t batch,
                                          int32_t cin, int32_t h, int32_t w_, int32_t cout,
                                          int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                                          void* stream) {
    int oh, ow;
    int rc = conv_common_check(nclients, batch, cin, h, w_, cout, kh, kw, stride, pad, oh, ow);
    if (rc) return rc;
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && sqnorm && workspace, "conv2d_persample_sqnorm: null pointer");
    const size_t need = fh_conv2d_persample_sqnorm_workspace(nclients, batch, cin, h, w_, cout, kh,
                                                             kw, stride, pad);
    FH_REQUIRE(ws_bytes >= need, "conv2d_persample_sqnorm: workspace %zu < %zu", ws_bytes, need);
    ConvArgs a = make_args(batch, cin, h, w_, cout, oh, ow, pad, counts);
    a.x = x; a.dy = dy; a.x_cs = x_cs; a.dy_cs = dy_cs;
    a.M = cout; a.N = cin * kh * kw; a.K = batch * oh * ow;
    const Plan p = plan_persample(a.M, a.N, oh * ow, batch);
    a.splits = batch;
    a.kchunk = oh * ow;
    a.sq_part = (float*)workspace;
    a.sq_bias = with_bias;
    hipStream_t st = as_stream(stream);
    dim3 grid((unsigned)ceil_div(a.N, p.t.bn), (unsigned)ceil_div(a.M, p.t.bm),
              (unsigned)(nclients * batch));
    rc = launch_shape<OP_WGRAD>(kh, kw, stride, p.t, grid, a, st);
    if (rc) return rc;
    FH_LAUNCH_CHECK("conv2d_persample_sqnorm");
    const int tiles = (int)(grid.x * grid.y);
    FH_LAUNCH(conv_sq_reduce_kernel, dim3((unsigned)ceil_div(batch, 256), nclients),
                       dim3(256), 0, st, (const float*)workspace, tiles, batch, counts, sqnorm);
    FH_LAUNCH_CHECK("conv2d_persample_sqnorm reduce");
    return FH_OK;
}


// ---- DP-SGD on the direct kernels (r04): per-image weight-gradient slabs -------------------
// The direct WGRAD kernels split their pixel reduction into slabs [z][split][cout*cin*9] (+ bias
// [z][split][cout] at wslab_bias_off); with one split per IMAGE the slab of split i is that
// image's own gradient dW_i (of the batch-mean loss, i.e. g_i / B).  One WGRAD pass then gives
// both what the clip needs — ||g_i||^2 = sum of squares of the image's slab rows, summed over
// the layers (fh_persample_slab_sqnorm) — and, once the clip coefficients c_i are known, the
// clipped sum sum_i c_i dW_i in image order (fh_persample_slab_wsum): no second WGRAD on rescaled
// dY and no implicit-GEMM norm tiles.  SimpleCNN: conv2 on the padded 16x16 planes
// (dwgrad_q_kernel, two 128-pixel stages = one image per split), conv1 from pool1's gradient
// (conv_c1_wgrad_mfma_kernel<POOLED>, seven 4-row stages = one 28x28 image per split).
constexpr int kC1PersampleNs4Max = 512;  // image workgroups: ~two per CU
static size_t persample_slab_bytes(int nclients, int batch, int per_w, int per_b) {
    return (size_t)wslab_bias_off(nclients, batch, per_w) +
           (size_t)nclients * batch * per_b * sizeof(float);
}

namespace fh {
// sqnorm[z][i] += sum_j w[z][i][j]^2 + sum_j b[z][i][j]^2 (fp64, one workgroup per (i, z),
// fixed order: per-thread strided partials, then block_sum_256)
__global__ void __launch_bounds__(256)
slab_sqnorm_kernel(const float* __restrict__ wpart, const float* __restrict__ bpart, int per_w,
                   int per_b, const int32_t* __restrict__ counts, int batch,
                   double* __restrict__ sqnorm) {
    __shared__ double red[4];
    const int i = blockIdx.x, z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    if (i >= cnt) return;  // block-uniform
    const int64_t row = (int64_t)z * batch + i;
    const float4* w4 = reinterpret_cast<const float4*>(wpart + row * per_w);
    double s = 0.0;
    for (int q = threadIdx.x; q < per_w / 4; q += 256) {
        const float4 v = w4[q];
        s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    if (bpart)
        for (int q = threadIdx.x; q < per_b; q += 256) {
            const double v = bpart[row * per_b + q];
            s += v * v;
        }
    s = block_sum_256(s, red);
    if (threadIdx.x == 0) sqnorm[row] += s;
}

// dw[z][j] = sum_{i < cnt} coef[z][i] * w[z][i][j] (float4 lanes; images in order, fl32
// multiply then add — -ffp-contract=off); the same for the bias slab into db
__global__ void __launch_bounds__(256)
slab_wsum_kernel(const float* __restrict__ wpart, const float* __restrict__ bpart, int per_w,
                 int per_b, const float* __restrict__ coef, const int32_t* __restrict__ counts,
                 int batch, float* __restrict__ dw, int64_t dw_cs, float* __restrict__ db,
                 int64_t db_cs) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const float* cz = coef + (int64_t)z * batch;
    const int q = blockIdx.x * 256 + threadIdx.x;
    const int nq = per_w / 4;
    if (q < nq) {
        const float4* w4 = reinterpret_cast<const float4*>(wpart + (int64_t)z * batch * per_w) + q;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int i = 0; i < cnt; ++i) {
            const float c = cz[i];
            const float4 v = w4[(int64_t)i * nq];
            acc.x = acc.x + c * v.x;
            acc.y = acc.y + c * v.y;
            acc.z = acc.z + c * v.z;
            acc.w = acc.w + c * v.w;
        }
        float* d = dw + z * dw_cs + 4 * q;
        d[0] = acc.x;
        d[1] = acc.y;
        d[2] = acc.z;
        d[3] = acc.w;
    } else if (bpart && db && q - nq < per_b) {
        const int j = q - nq;
        float acc = 0.f;
        for (int i = 0; i < cnt; ++i) acc = acc + cz[i] * bpart[((int64_t)z * batch + i) * per_b + j];
        db[z * db_cs + j] = acc;
    }
}
}  // namespace fh

extern "C" size_t fh_conv2d_wgrad_persample_workspace(int32_t nclients, int32_t batch,
                                                      int32_t cin, int32_t cout) {
    if (nclients <= 0 || batch <= 0) return 0;
    return persample_slab_bytes(nclients, batch, cout * cin * 9, cout);
}

extern "C" int fh_conv2d_wgrad_persample(const float* x, int64_t x_cs, const float* dy,
                                         int64_t dy_cs, void* slab, size_t slab_bytes,
                                         const int32_t* counts, int32_t nclients, int32_t batch,
                                         int32_t cin, int32_t h, int32_t w_, int32_t cout,
                                         void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0, "conv2d_wgrad_persample: bad shape");
    FH_REQUIRE(dwgrad_supported(cin, cout, h, w_, 3, 3, 1, 1),
               "conv2d_wgrad_persample: 3x3/s1/p1 on a square 8/16/32 map, channels %% 32 "
               "(got cin %d cout %d %dx%d)", cin, cout, h, w_);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && slab, "conv2d_wgrad_persample: null pointer");
    FH_REQUIRE((uintptr_t)x % 16 == 0 && (uintptr_t)dy % 16 == 0 && x_cs % 4 == 0 &&
               dy_cs % 4 == 0, "conv2d_wgrad_persample: x / dy must be 16-B aligned");
    const size_t need = fh_conv2d_wgrad_persample_workspace(nclients, batch, cin, cout);
    FH_REQUIRE(slab_bytes >= need, "conv2d_wgrad_persample: slab %zu < %zu", slab_bytes, need);
    const int N = cin * 9;
    DWArgs d{};
    d.x = x; d.dy = dy; d.x_cs = x_cs; d.dy_cs = dy_cs; d.counts = counts;
    d.batch = batch; d.cin = cin; d.M = cout; d.N = N;
    d.splits = batch;                                      // one split per image
    const int spx = w_ == 8 ? 64 : 128;                    // a stage never straddles two images
    d.stages_per_split = (w_ * w_) / spx;
    d.part = (float*)slab;
    d.bias_part = (float*)((char*)slab + wslab_bias_off(nclients, batch, cout * N));
    hipStream_t st = as_stream(stream);
    const dim3 grid((unsigned)batch, (unsigned)((cout / 32) * (cin / 32)), (unsigned)nclients);
    // fh_conv_pair armed (r05, DP-SGD's conv2): the slabs need no reduction launch, so the launch
    // is held for the layer's DGRAD like a training step's deferred WGRAD (one dual-role grid),
    // with an armed pooled dY (fh_conv_pooled_dy) travelling along
    const int pair = g_pair_mode;
    g_pair_mode = 0;
    const bool hold = pair && w_ != 8;
    if (g_pdy.on && !g_pdy.done && !(hold && w_ == 16)) {
        const int rc = pdy_materialize(const_cast<float*>(dy), dy_cs, counts, nclients, batch, cout,
                                       w_, st);
        if (rc) return rc;
    }
    if (hold) {
        if (const int fr = flush_pending_wgrad()) return fr;
        g_pend.w = w_;
        g_pend.mode = pair;
        g_pend.grid = grid;
        g_pend.d = d;
        g_pend.st = st;
        g_pend.on = true;
        g_pend.pdy = g_pdy.on && !g_pdy.done && w_ == 16;
        if (g_pend.pdy) g_pend.d.pdy = g_pdy.p;
        return FH_OK;
    }
    if (w_ == 32) FH_LAUNCH((dwgrad_q_kernel<32, 128, false>), grid, dim3(256), 0, st, d);
    else if (w_ == 16) FH_LAUNCH((dwgrad_q_kernel<16, 128, false>), grid, dim3(256), 0, st, d);
    else FH_LAUNCH((dwgrad_q_kernel<8, 64, true>), grid, dim3(256), 0, st, d);
    FH_LAUNCH_CHECK("conv2d_wgrad_persample");
    return FH_OK;
}

static int c1_persample_impl(const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs,
                             const uint8_t* idx, int64_t i_cs, const float* y, int64_t y_cs,
                             void* slab, size_t slab_bytes, const int32_t* counts,
                             int32_t nclients, int32_t batch, int32_t h, int32_t w_, int32_t cout,
                             int32_t gh, int32_t gw, const NormTail* tail, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && h % 4 == 0 && w_ % 4 == 0 && w_ <= 32 &&
               gh >= h / 2 && gw >= w_ / 2, "conv2d_c1_pool_wgrad_persample: bad shape");
    FH_REQUIRE(cout == 32 || cout == 64, "conv2d_c1_pool_wgrad_persample: cout %d (32 or 64)", cout);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dpool && idx && y && slab, "conv2d_c1_pool_wgrad_persample: null pointer");
    FH_REQUIRE((uintptr_t)x % 16 == 0 && x_cs % 4 == 0,
               "conv2d_c1_pool_wgrad_persample: x must be 16-B aligned");
    const size_t need = fh_conv2d_wgrad_persample_workspace(nclients, batch, 1, cout);
    FH_REQUIRE(slab_bytes >= need, "conv2d_c1_pool_wgrad_persample: slab %zu < %zu", slab_bytes,
               need);
    float* part = (float*)slab;
    float* bpart = (float*)((char*)slab + wslab_bias_off(nclients, batch, cout * 9));
    const int sps = h / 4;  // one image per split
    const dim3 grid((unsigned)batch, (unsigned)nclients);
    hipStream_t st = as_stream(stream);
    // narrow grids (fewer image workgroups than ~two per CU): four stages per LDS round
    const bool wide4 = (int64_t)batch * nclients <= kC1PersampleNs4Max;
    const NormTail t = tail ? *tail : NormTail{};
    DgradParts dpa{};  // a deferred DGRAD reduction of dpool: summed while staging (cout 32)
    if (const int rc = ddef_take(dpool, dp_cs, gh, gw, st, dpa)) return rc;
    if (dpa.p && cout != 32) {
        g_ddef.pending = true;
        if (const int rc = ddef_materialize()) return rc;
        dpa = DgradParts{};
    }
#define FH_C1PS(CO, NS, NORM, NP)                                                                \
    FH_LAUNCH((conv_c1_wgrad_mfma_kernel<CO, true, NS, NORM, NP>), grid, dim3(256), 0, st, x,   \
              x_cs, dpool, dp_cs, part, bpart, counts, batch, h, w_, batch, sps, idx, i_cs, y,   \
              y_cs, gh, gw, t, dpa)
    if (tail) {
        FH_REQUIRE(cout == 32, "conv2d_c1_pool_wgrad_persample_clip: cout 32 (got %d)", cout);
        if (dpa.p) FH_C1PS(32, 2, true, kDgradPartsMax);
        else if (wide4) FH_C1PS(32, 4, true, 0);
        else FH_C1PS(32, 2, true, 0);
    } else if (cout == 32) {
        if (dpa.p) FH_C1PS(32, 2, false, kDgradPartsMax);
        else if (wide4) FH_C1PS(32, 4, false, 0);
        else FH_C1PS(32, 2, false, 0);
    } else {
        FH_C1PS(64, 2, false, 0);
    }
#undef FH_C1PS
    FH_LAUNCH_CHECK("conv2d_c1_pool_wgrad_persample");
    return FH_OK;
}

extern "C" int fh_conv2d_c1_pool_wgrad_persample(const float* x, int64_t x_cs, const float* dpool,
                                                 int64_t dp_cs, const uint8_t* idx, int64_t i_cs,
                                                 const float* y, int64_t y_cs, void* slab,
                                                 size_t slab_bytes, const int32_t* counts,
                                                 int32_t nclients, int32_t batch, int32_t h,
                                                 int32_t w_, int32_t cout, int32_t gh, int32_t gw,
                                                 void* stream) {
    return c1_persample_impl(x, x_cs, dpool, dp_cs, idx, i_cs, y, y_cs, slab, slab_bytes, counts,
                             nclients, batch, h, w_, cout, gh, gw, nullptr, stream);
}

static int norm_srcs(const fh_linear_norm_src* lin, int32_t nlin, const fh_slab_norm_src* slabs,
                     int32_t nslab, int32_t nclients, int32_t batch, NormSrcs& s) {
    FH_REQUIRE(nlin >= 0 && nlin <= kNormSrcMax && nslab >= 0 && nslab <= kNormSrcMax,
               "dpsgd_norm_clip: bad shape (%d linear, %d slab sources)", nlin, nslab);
    FH_REQUIRE((nlin == 0 || lin) && (nslab == 0 || slabs), "dpsgd_norm_clip: null pointer");
    s = NormSrcs{};
    s.nlin = nlin;
    for (int l = 0; l < nlin; ++l) {
        FH_REQUIRE(lin[l].x && lin[l].dy && lin[l].in_f > 0 && lin[l].out_f > 0,
                   "dpsgd_norm_clip: bad linear source %d", l);
        s.lin[l] = lin[l];
    }
    s.nslab = nslab;
    for (int l = 0; l < nslab; ++l) {
        FH_REQUIRE(slabs[l].slab && slabs[l].per_w > 0 && slabs[l].per_w % 4 == 0 &&
                       slabs[l].per_b >= 0 && (uintptr_t)slabs[l].slab % 16 == 0,
                   "dpsgd_norm_clip: bad slab source %d", l);
        s.sw[l] = (const float*)slabs[l].slab;
        s.sb[l] = slabs[l].per_b ? (const float*)((const char*)slabs[l].slab +
                                                  wslab_bias_off(nclients, batch, slabs[l].per_w))
                                 : nullptr;
        s.per_w[l] = slabs[l].per_w;
        s.per_b[l] = slabs[l].per_b;
    }
    return FH_OK;
}

extern "C" int fh_dpsgd_norm_clip(const fh_linear_norm_src* lin, int32_t nlin,
                                  const fh_slab_norm_src* slabs, int32_t nslab,
                                  const int32_t* counts, int32_t nclients, int32_t batch,
                                  double max_norm, double* sqnorm, float* coef, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0, "dpsgd_norm_clip: bad shape");
    FH_REQUIRE(max_norm > 0.0, "dpsgd_norm_clip: max_norm must be > 0");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(coef, "dpsgd_norm_clip: null pointer");
    NormSrcs s;
    if (const int rc = norm_srcs(lin, nlin, slabs, nslab, nclients, batch, s)) return rc;
    FH_LAUNCH(dpsgd_norm_clip_kernel, dim3((unsigned)batch, (unsigned)nclients), dim3(256), 0,
              as_stream(stream), s, counts, batch, max_norm, sqnorm, coef);
    FH_LAUNCH_CHECK("dpsgd_norm_clip");
    return FH_OK;
}

// fh_conv2d_c1_pool_wgrad_persample + fh_dpsgd_norm_clip in ONE launch (r05): the per-image
// conv1 slab workgroup (one per image and client, the norm launch's grid) finishes with the
// image's norm over the given sources — which must include this launch's own slab — and its
// clip coefficient, the same code and sums as fh_dpsgd_norm_clip.  cout 32.
extern "C" int fh_conv2d_c1_pool_wgrad_persample_clip(
        const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs, const uint8_t* idx,
        int64_t i_cs, const float* y, int64_t y_cs, void* slab, size_t slab_bytes,
        const int32_t* counts, int32_t nclients, int32_t batch, int32_t h, int32_t w_,
        int32_t cout, int32_t gh, int32_t gw, const fh_linear_norm_src* lin, int32_t nlin,
        const fh_slab_norm_src* slabs, int32_t nslab, double max_norm, double* sqnorm,
        float* coef, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0, "conv2d_c1_pool_wgrad_persample_clip: bad shape");
    FH_REQUIRE(max_norm > 0.0, "conv2d_c1_pool_wgrad_persample_clip: max_norm must be > 0");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(coef, "conv2d_c1_pool_wgrad_persample_clip: null pointer");
    bool own = false;
    for (int l = 0; l < nslab && slabs; ++l) own = own || slabs[l].slab == slab;
    FH_REQUIRE(own, "conv2d_c1_pool_wgrad_persample_clip: the slab sources must include this "
                    "launch's own slab");
    NormTail t{};
    if (const int rc = norm_srcs(lin, nlin, slabs, nslab, nclients, batch, t.src)) return rc;
    t.max_norm = max_norm;
    t.sqnorm = sqnorm;
    t.coef = coef;
    return c1_persample_impl(x, x_cs, dpool, dp_cs, idx, i_cs, y, y_cs, slab, slab_bytes, counts,
                             nclients, batch, h, w_, cout, gh, gw, &t, stream);
}

extern "C" int fh_persample_slab_sqnorm(const void* slab, int32_t per_w, int32_t per_b,
                                        const int32_t* counts, int32_t nclients, int32_t batch,
                                        double* sqnorm, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && per_w > 0 && per_w % 4 == 0 && per_b >= 0,
               "persample_slab_sqnorm: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(slab && sqnorm, "persample_slab_sqnorm: null pointer");
    const float* w = (const float*)slab;
    const float* b = per_b ? (const float*)((const char*)slab + wslab_bias_off(nclients, batch, per_w))
                           : nullptr;
    FH_LAUNCH(slab_sqnorm_kernel, dim3((unsigned)batch, (unsigned)nclients), dim3(256), 0,
              as_stream(stream), w, b, per_w, per_b, counts, batch, sqnorm);
    FH_LAUNCH_CHECK("persample_slab_sqnorm");
    return FH_OK;
}

extern "C" int fh_persample_slab_wsum(const void* slab, int32_t per_w, int32_t per_b,
                                      const float* coef, const int32_t* counts, int32_t nclients,
                                      int32_t batch, float* dw, int64_t dw_cs, float* db,
                                      int64_t db_cs, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && per_w > 0 && per_w % 4 == 0 && per_b >= 0,
               "persample_slab_wsum: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(slab && coef && dw, "persample_slab_wsum: null pointer");
    FH_REQUIRE(!per_b || db, "persample_slab_wsum: bias slab without db");
    const float* w = (const float*)slab;
    const float* b = per_b ? (const float*)((const char*)slab + wslab_bias_off(nclients, batch, per_w))
                           : nullptr;
    const int threads = per_w / 4 + per_b;
    FH_LAUNCH(slab_wsum_kernel, dim3((unsigned)ceil_div(threads, 256), (unsigned)nclients),
              dim3(256), 0, as_stream(stream), w, b, per_w, per_b, coef, counts, batch, dw, dw_cs,
              db, db_cs);
    FH_LAUNCH_CHECK("persample_slab_wsum");
    return FH_OK;
}
