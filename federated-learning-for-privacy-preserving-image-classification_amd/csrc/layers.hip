// layers.hip — the non-GEMM layers of the reference CNNs, client-batched.
//
//   (BatchNorm2d lives in bn.hip)
//   MaxPool2d(2,2) fwd/bwd              models_pytorch.py:72, 123 (fused with the Dropout
//       that follows it in CIFAR10CNN, :139-155, and the ReLU before it in SimpleCNN, :85-88)
//   Dropout fwd/bwd                     models_pytorch.py:75, 124 (F.dropout semantics:
//       y = x * (bernoulli(1-p) / (1-p)), training-mode only)
//   CrossEntropyLoss fwd+bwd + metrics  training.py:90, 193, 200-203
//   AdaptiveAvgPool2d((1,1))            models_pytorch.py:216, 241
//   batch gather                        DataLoader(batch_size=32, shuffle=True) data path
//
// Every kernel takes per-client valid image counts: reductions (BN stats, loss,
// gradients) cover only valid images; invalid rows are never read by a reduction.
// All per-(client, channel) reductions accumulate in fp64, as ATen's CPU
// batch-norm does (acc_type<float> on CPU is double).
#include "fh_common.h"

namespace fh {

typedef float hf32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ MaxPool 2x2 (+dropout)
// x: [z][img][C][H][W] -> y: [z][img][C][H/2][W/2]; idx: window argmax (0..3, first max);
// drop_mode 0: none; 1: generate keep-mask (Philox) into mask; 2: use caller mask.
__global__ void __launch_bounds__(256)
maxpool2_fwd_kernel(const float* __restrict__ x, int64_t x_cs, float* __restrict__ y,
                    int64_t y_cs, uint8_t* __restrict__ idx, int64_t i_cs,
                    uint8_t* __restrict__ mask, int64_t m_cs, const int32_t* __restrict__ counts,
                    int batch, int C, int H, int W, int drop_mode, float keep_prob, float scale,
                    uint64_t seed_salt, const uint64_t* __restrict__ seed_dev,
                    const float* __restrict__ in_scale, const float* __restrict__ in_shift,
                    int64_t aff_cs, int xh, int xw, int yh, int yw) {
    // x planes are xh x xw (row pitch xw) holding the H x W map in their top-left corner,
    // y planes yh x yw holding the pooled map likewise (a map embedded in a wider zero
    // ring for the direct-conv kernels); idx / mask stay dense [img][C][H/2][W/2]
    const uint64_t seed = seed_salt + (seed_dev ? *seed_dev : 0ull);
    const int z = blockIdx.y;
    const uint64_t prow = drop_mode == 1 ? philox_row(seed_dev, z) : 0ull;  // once, not per store
    const int cnt = counts ? counts[z] : batch;
    const int OH = H / 2, OW = W / 2;
    // 32-bit unsigned index arithmetic (a client's batch is < 2^31 elements; the 64-bit
    // divisions cost more than the pool itself)
    const uint32_t per_img = (uint32_t)(C * OH * OW);
    const uint32_t total = (uint32_t)cnt * per_img;
    const float* xb = x + z * x_cs;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += gridDim.x * blockDim.x) {
        const uint32_t t = e / (uint32_t)OW;
        const int ow = (int)(e - t * (uint32_t)OW);
        const uint32_t plane = t / (uint32_t)OH;  // img*C + c
        const int oh = (int)(t - plane * (uint32_t)OH);
        const float* p = xb + (int64_t)plane * xh * xw + (2 * oh) * xw + 2 * ow;
        float v0 = p[0], v1 = p[1], v2 = p[xw], v3 = p[xw + 1];
        if (in_scale) {  // input = BN pre-activation: relu(x*scale + shift), bn_apply's ops
            const int c = (int)(plane % C);
            const float s = in_scale[z * aff_cs + c], t = in_shift[z * aff_cs + c];
            v0 = fmaxf(v0 * s + t, 0.f);
            v1 = fmaxf(v1 * s + t, 0.f);
            v2 = fmaxf(v2 * s + t, 0.f);
            v3 = fmaxf(v3 * s + t, 0.f);
        }
        float m = v0;
        int a = 0;
        if (v1 > m) { m = v1; a = 1; }
        if (v2 > m) { m = v2; a = 2; }
        if (v3 > m) { m = v3; a = 3; }
        idx[z * i_cs + e] = (uint8_t)a;
        if (drop_mode) {
            uint8_t keep;
            if (drop_mode == 1) {
                const uint4 r = Philox::gen(seed, prow, (uint64_t)e);
                keep = u01(r.x) <= keep_prob ? 1 : 0;
                mask[z * m_cs + e] = keep;
            } else {
                keep = mask[z * m_cs + e];
            }
            m = keep ? m * scale : 0.f;
        }
        y[z * y_cs + (int64_t)plane * yh * yw + oh * yw + ow] = m;
    }
}

// dx (all 4 window slots written) = dy routed to the argmax, times the dropout
// factor; relu_in: also zero where the pooled input (a ReLU output) is not > 0.
__global__ void __launch_bounds__(256)
maxpool2_bwd_kernel(const float* __restrict__ dy, int64_t dy_cs, const uint8_t* __restrict__ idx,
                    int64_t i_cs, const uint8_t* __restrict__ mask, int64_t m_cs,
                    const float* __restrict__ xin, int64_t x_cs, float* __restrict__ dx,
                    int64_t dx_cs, const int32_t* __restrict__ counts, int batch, int C, int H,
                    int W, float scale, int gh, int gw, int xh, int xw,
                    const float* __restrict__ yin, int64_t yin_cs) {
    // yin (nullable): the pooled ReLU output (planes gh x gw) — the ReLU mask at the argmax
    // is yin > 0, the same decision as xin at the argmax (that IS the pooled value), for a
    // forward that never wrote the full-resolution xin (fh_conv2d_c1_pool_fwd)
    // dy planes gh x gw, dx / xin planes xh x xw (maps in the top-left corner, see
    // maxpool2_fwd_kernel); idx / mask dense
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int OH = H / 2, OW = W / 2;
    const uint32_t total = (uint32_t)cnt * (uint32_t)(C * OH * OW);  // 32-bit: see the fwd
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += gridDim.x * blockDim.x) {
        const uint32_t t = e / (uint32_t)OW;
        const int ow = (int)(e - t * (uint32_t)OW);
        const uint32_t pl = t / (uint32_t)OH;
        const int oh = (int)(t - pl * (uint32_t)OH);
        const int64_t plane = pl;
        float g = dy[z * dy_cs + plane * gh * gw + oh * gw + ow];
        if (mask) g = mask[z * m_cs + e] ? g * scale : 0.f;
        const int a = idx[z * i_cs + e];
        const int64_t base = plane * xh * xw + (2 * oh) * xw + 2 * ow;
        const int64_t off[4] = {0, 1, xw, xw + 1};
        if (xin && !(xin[z * x_cs + base + off[a]] > 0.f)) g = 0.f;
        if (yin && !(yin[z * yin_cs + plane * gh * gw + oh * gw + ow] > 0.f)) g = 0.f;
        float* d = dx + z * dx_cs + base;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[off[q]] = (q == a) ? g : 0.f;
    }
}

// ------------------------------------------------------------------ Dropout (+ReLU mask)
__global__ void __launch_bounds__(256)
dropout_fwd_kernel(const float* __restrict__ x, int64_t x_cs, float* __restrict__ y, int64_t y_cs,
                   uint8_t* __restrict__ mask, int64_t m_cs, const int32_t* __restrict__ counts,
                   int batch, int64_t per_img, int drop_mode, float keep_prob, float scale,
                   uint64_t seed_salt, const uint64_t* __restrict__ seed_dev) {
    const uint64_t seed = seed_salt + (seed_dev ? *seed_dev : 0ull);
    const int z = blockIdx.y;
    const uint64_t prow = drop_mode == 1 ? philox_row(seed_dev, z) : 0ull;  // once, not per store
    const int cnt = counts ? counts[z] : batch;
    const int64_t total = cnt * per_img;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        uint8_t keep;
        if (drop_mode == 1) {
            const uint4 r = Philox::gen(seed, prow, (uint64_t)e);
            keep = u01(r.x) <= keep_prob ? 1 : 0;
            mask[z * m_cs + e] = keep;
        } else {
            keep = mask[z * m_cs + e];
        }
        const float v = x[z * x_cs + e];
        y[z * y_cs + e] = keep ? v * scale : 0.f;
    }
}

// dx = dy * mask * scale [* (relu_out > 0)]; mask may be NULL (pure ReLU backward).
__global__ void __launch_bounds__(256)
dropout_bwd_kernel(const float* __restrict__ dy, int64_t dy_cs, const uint8_t* __restrict__ mask,
                   int64_t m_cs, const float* __restrict__ relu_out, int64_t r_cs,
                   float* __restrict__ dx, int64_t dx_cs, const int32_t* __restrict__ counts,
                   int batch, int64_t per_img, float scale) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int64_t total = cnt * per_img;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        float g = dy[z * dy_cs + e];
        if (mask) g = mask[z * m_cs + e] ? g * scale : 0.f;
        if (relu_out && !(relu_out[z * r_cs + e] > 0.f)) g = 0.f;
        dx[z * dx_cs + e] = g;
    }
}

// ------------------------------------------------------------------ CrossEntropy
// One block per client.  logits/dlogits: [z][img][K]; targets: int64 [z][img].
// loss_out[z] = batch-mean loss (fp32, = loss.item()); accumulators (may be NULL):
// acc_loss[z] += loss_out[z] (double), acc_correct[z] += #argmax==target, acc_seen[z] += cnt.
__global__ void __launch_bounds__(256)
ce_kernel(const float* __restrict__ logits, int64_t l_cs, const int64_t* __restrict__ targets,
          int64_t t_cs, float* __restrict__ dlogits, int64_t d_cs, float* __restrict__ loss_out,
          double* __restrict__ acc_loss, int64_t* __restrict__ acc_correct,
          int64_t* __restrict__ acc_seen, const int32_t* __restrict__ reset,
          const int32_t* __restrict__ counts, int batch, int K) {
    __shared__ double sl[4];
    __shared__ int sc[4];
    __shared__ double li[256];
    __shared__ int ci[256];
    const int z = blockIdx.x;
    const int cnt = counts ? counts[z] : batch;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double lsum = 0.0;
    int corr = 0;
    const float inv_n = cnt > 0 ? 1.0f / (float)cnt : 0.f;
    if (K <= 16 && cnt <= 256) {
        // 16 lanes per image, 16 images at once (a batch of 32 in two passes instead of
        // eight wave-serial ones); per-image losses go through LDS so the fp64 sums below
        // run in exactly the order of the wave-per-image path
        const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
        for (int img = g; img < cnt; img += 16) {
            const float* row = logits + z * l_cs + (int64_t)img * K;
            const int tgt = (int)targets[z * t_cs + img];
            const float v = l < K ? row[l] : -INFINITY;
            float mx = v;
            int amax = l < K ? l : K;
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {  // first index of the max (torch.max tie rule)
                const float om = __shfl_xor(mx, o, 16);
                const int oa = __shfl_xor(amax, o, 16);
                if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
            }
            float se = l < K ? expf(v - mx) : 0.f;
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) se += __shfl_xor(se, o, 16);
            const float lse = logf(se);
            if (l == 0) {
                li[img] = (double)(-((row[tgt] - mx) - lse));
                ci[img] = amax == tgt;
            }
            if (l < K) {
                const float p = expf((v - mx) - lse);
                dlogits[z * d_cs + (int64_t)img * K + l] = (p - (l == tgt ? 1.f : 0.f)) * inv_n;
            }
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            for (int img = threadIdx.x; img < cnt; img += 4) {
                lsum += li[img];
                corr += ci[img];
            }
            sl[threadIdx.x] = lsum;
            sc[threadIdx.x] = corr;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const double tot = sl[0] + sl[1] + sl[2] + sl[3];
            const float batch_loss = cnt > 0 ? (float)(tot / (double)cnt) : 0.f;
            const bool rs = reset && reset[z];
            if (loss_out) loss_out[z] = batch_loss;
            if (acc_loss) acc_loss[z] = (rs ? 0.0 : acc_loss[z]) + (double)batch_loss;
            if (acc_correct) acc_correct[z] = (rs ? 0 : acc_correct[z]) + sc[0] + sc[1] + sc[2] + sc[3];
            if (acc_seen) acc_seen[z] = (rs ? 0 : acc_seen[z]) + cnt;
        }
        return;
    }
    for (int img = wid; img < cnt; img += 4) {
        const float* row = logits + z * l_cs + (int64_t)img * K;
        const int tgt = (int)targets[z * t_cs + img];
        float mx = -INFINITY;
        int amax = 0;
        for (int k = lane; k < K; k += 64) {
            const float v = row[k];
            if (v > mx) { mx = v; amax = k; }
        }
        // first index of the max (torch.max tie rule)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float om = __shfl_xor(mx, o, 64);
            const int oa = __shfl_xor(amax, o, 64);
            if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
        }
        float se = 0.f;
        for (int k = lane; k < K; k += 64) se += expf(row[k] - mx);
        se = wave_sum(se);
        const float lse = logf(se);
        // loss_i = -(x_t - mx - lse)
        if (lane == 0) {
            lsum += (double)(-((row[tgt] - mx) - lse));
            corr += (amax == tgt);
        }
        float* drow = dlogits + z * d_cs + (int64_t)img * K;
        for (int k = lane; k < K; k += 64) {
            const float p = expf((row[k] - mx) - lse);
            drow[k] = (p - (k == tgt ? 1.f : 0.f)) * inv_n;
        }
    }
    if (lane == 0) {
        sl[wid] = lsum;
        sc[wid] = corr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double tot = sl[0] + sl[1] + sl[2] + sl[3];
        const float batch_loss = cnt > 0 ? (float)(tot / (double)cnt) : 0.f;
        const bool rs = reset && reset[z];
        if (loss_out) loss_out[z] = batch_loss;
        if (acc_loss) acc_loss[z] = (rs ? 0.0 : acc_loss[z]) + (double)batch_loss;
        if (acc_correct) acc_correct[z] = (rs ? 0 : acc_correct[z]) + sc[0] + sc[1] + sc[2] + sc[3];
        if (acc_seen) acc_seen[z] = (rs ? 0 : acc_seen[z]) + cnt;
    }
}

// ------------------------------------------------------------------ classifier head
// The end of a training step's forward and the start of its backward in ONE launch (S
// blocks per client): the last linear layer (logits = x W^T + b: CIFAR10CNN fc3
// models_pytorch.py:159-165, SimpleCNN fc2 :96-97, FederatedResNet fc :241-246), the
// cross-entropy forward + backward with ce_kernel's arithmetic and accumulators
// (training.py:193-203), the layer's weight and bias gradients, and the gradient of its
// input through the Dropout (keep-mask, scale 1/(1-p)) and ReLU in front of it — ReLU
// decided on the layer input itself (x > 0 <=> the pre-dropout ReLU output > 0 wherever
// the keep-mask is 1; elsewhere the gradient is 0 anyway).  Replaces the layer's forward
// (+ split-K epilogue), ce, its wgrad, its dgrad and dropout_bwd.  batch <= 32.
// Every block of a client stages x [cnt][F] (and, SMALLK, W [K][F]) in LDS with a +1 pitch,
// recomputes the logits and the loss, and then owns 1/S of the dW and dX outputs; block 0
// publishes logits, dlogits and the loss accumulators.  SMALLK (<= 16 classes, F <= 256, the
// BASELINE models' heads): the three products run on v_mfma_f32_16x16x4_f32 from the staged
// LDS operands — logits as two 16-image tiles x two halves of F (one wave each), dW / dX as
// 16-column tiles dealt round-robin to the S x 4 waves of the client (r04: the per-thread
// fmaf chains made the launch ~20 us of dependent LDS round trips); else sequential fmaf
// chains (one thread per output), images / classes in order.
constexpr int kHeadBlocks = 4;
template <bool SMALLK>
__global__ void __launch_bounds__(256)
linear_head_ce_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ w,
                      int64_t w_cs, const float* __restrict__ bias, int64_t b_cs,
                      const int64_t* __restrict__ targets, int64_t t_cs, float* __restrict__ logits,
                      int64_t l_cs, float* __restrict__ dlogits, int64_t d_cs,
                      float* __restrict__ loss_out, double* __restrict__ acc_loss,
                      int64_t* __restrict__ acc_correct, int64_t* __restrict__ acc_seen,
                      const int32_t* __restrict__ reset, float* __restrict__ dw, int64_t dw_cs,
                      float* __restrict__ db, int64_t db_cs, float* __restrict__ dx,
                      int64_t dx_cs, const uint8_t* __restrict__ mask, int64_t m_cs, float scale,
                      int relu_in, const int32_t* __restrict__ counts, int batch, int F, int K) {
    constexpr int KMAX = SMALLK ? 16 : 128;
    constexpr int FMAX = 256;                      // SMALLK: staged x / W width (F <= 256)
    constexpr int XS = SMALLK ? 32 * (FMAX + 1) : 1;
    constexpr int WS = SMALLK ? KMAX * (FMAX + 1) : 1;
    __shared__ float Xs[XS];
    __shared__ float Ws[WS];
    __shared__ float L[32 * KMAX];   // logits [img][K]
    __shared__ float D[32 * KMAX];   // dlogits [img][K]
    __shared__ double li[32];
    __shared__ int ci[32];
    __shared__ double sl[4];
    __shared__ int sc[4];
    // SMALLK: the targets, the bias and the keep-mask, fetched with the operands at the
    // start (r04: loaded where used they were three more dependent global round trips)
    constexpr int MS = SMALLK ? 32 * FMAX : 1;
    __shared__ int64_t Ts[32];
    __shared__ float Bs[KMAX];
    __shared__ uint8_t Ms[MS];
    const int z = blockIdx.y, part = blockIdx.x, tid = threadIdx.x;
    const int cnt = counts ? counts[z] : batch;
    const float* xz = x + z * x_cs;
    const float* wz = w + z * w_cs;
    const int FP = F + 1;
    const int S = gridDim.x;
    // block 0, thread 0: the running accumulators it updates at the end (SMALLK: loaded after
    // the operands' loads are issued)
    bool rs0 = false;
    double al0 = 0.0;
    int64_t ac0 = 0, as0 = 0;
    auto load_acc = [&]() {
        if (part == 0 && tid == 0) {
            rs0 = reset && reset[z];
            if (acc_loss) al0 = acc_loss[z];
            if (acc_correct) ac0 = acc_correct[z];
            if (acc_seen) as0 = acc_seen[z];
        }
    };
    const int dx_per = (cnt * F + S - 1) / S, dx_e0 = part * dx_per;
    const int dx_e1 = min(cnt * F, dx_e0 + dx_per);
    if constexpr (SMALLK) {
        // every global load of the prologue is issued before the first LDS store: the targets,
        // the bias, the keep-mask words, x and W, then the accumulators (r05: each section's
        // store waited for its own loads before the next section's loads were issued — four
        // dependent global round trips; r03 / r04 had removed those inside the sections)
        const int64_t tv = tid < cnt ? targets[z * t_cs + tid] : 0;
        const float bv = (tid < K && bias) ? bias[z * b_cs + tid] : 0.f;
        const uint8_t* mz = mask + z * m_cs;
        const bool mwords = mask && dx && ((uintptr_t)mz & 3) == 0;  // cnt * F % 16 == 0
        constexpr int NM = 32 * FMAX / 4 / 256;
        uint32_t mw[NM];
        if (mwords) {
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                const int e = tid + 256 * i;
                mw[i] = e < cnt * F / 4 ? reinterpret_cast<const uint32_t*>(mz)[e] : 0u;
            }
        }
        const bool v4 = (F & 3) == 0 && ((uintptr_t)xz & 15) == 0 && ((uintptr_t)wz & 15) == 0;
        constexpr int NX = 32 * FMAX / 4 / 256, NW = KMAX * FMAX / 4 / 256;
        const int F4 = F / 4;
        float4 xv[NX], wv[NW];
        if (v4) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const int e4 = tid + 256 * i;
                xv[i] = e4 < cnt * F4 ? *reinterpret_cast<const float4*>(xz + 4 * e4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int e4 = tid + 256 * i;
                wv[i] = e4 < K * F4 ? *reinterpret_cast<const float4*>(wz + 4 * e4)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        load_acc();
        if (tid < cnt) Ts[tid] = tv;
        if (tid < K) Bs[tid] = bv;
        if (mwords) {
#pragma unroll
            for (int i = 0; i < NM; ++i) {
                const int e = tid + 256 * i;
                if (e < cnt * F / 4) reinterpret_cast<uint32_t*>(Ms)[e] = mw[i];
            }
        } else if (mask && dx) {
            for (int e = tid; e < cnt * F; e += 256) Ms[e] = mz[e];
        }
        if (v4) {
#pragma unroll
            for (int i = 0; i < NX; ++i) {
                const int e4 = tid + 256 * i;
                if (e4 < cnt * F4) {
                    const int b = e4 / F4, f = 4 * (e4 - b * F4);
                    float* d = Xs + b * FP + f;
                    d[0] = xv[i].x; d[1] = xv[i].y; d[2] = xv[i].z; d[3] = xv[i].w;
                }
            }
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int e4 = tid + 256 * i;
                if (e4 < K * F4) {
                    const int k = e4 / F4, f = 4 * (e4 - k * F4);
                    float* d = Ws + k * FP + f;
                    d[0] = wv[i].x; d[1] = wv[i].y; d[2] = wv[i].z; d[3] = wv[i].w;
                }
            }
        } else {
            for (int e = tid; e < cnt * F; e += 256) {
                const int b = e / F;
                Xs[b * FP + (e - b * F)] = xz[e];
            }
            for (int e = tid; e < K * F; e += 256) {
                const int k = e / F;
                Ws[k * FP + (e - k * F)] = wz[e];
            }
        }
        __syncthreads();
    } else {
        load_acc();
    }
    auto X = [&](int b, int f) -> float { return SMALLK ? Xs[b * FP + f] : xz[(int64_t)b * F + f]; };
    auto Wt = [&](int k, int f) -> float { return SMALLK ? Ws[k * FP + f] : wz[(int64_t)k * F + f]; };
    // 1. logits
    const int lane = tid & 63, wid = tid >> 6;
    if constexpr (SMALLK) {
        // wave wid: image tile t (16 rows), half fh of F; D [img][16] holds the second half's
        // partial products until the CE pass
        const int mn = lane & 15, kk = lane >> 4, t = wid & 1, fh = wid >> 1, Fh = F >> 1;
        const int ia = t * 16 + mn;
        const bool arow = ia < cnt, bcol = mn < K;
        const float* xa = Xs + ia * FP + fh * Fh + kk;
        const float* wb = Ws + mn * FP + fh * Fh + kk;
        // r06: every operand read up front (unconditional: the arrays hold FMAX-wide rows, so
        // any F <= FMAX stays in bounds; past Fh the values are unused), then the MFMA chain in
        // the same order — the read -> MFMA loop waited on each pair, ~2.5 us of the launch
        constexpr int NQ = FMAX / 8;
        float xr[NQ], wr[NQ];
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
            const float xv = xa[4 * u], wv2 = wb[4 * u];
            xr[u] = arow ? xv : 0.f;
            wr[u] = bcol ? wv2 : 0.f;
        }
        hf32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < NQ; ++u)
            if (4 * u < Fh) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[u], wr[u], acc, 0, 0, 0);
        float* lp = fh ? D : L;
#pragma unroll
        for (int r = 0; r < 4; ++r) lp[(t * 16 + 4 * kk + r) * 16 + mn] = acc[r];
        __syncthreads();
        float lv[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int o = tid + 256 * u;
            const int img = o / K, k = o - img * K;
            lv[u] = o < cnt * K ? L[img * 16 + k] + D[img * 16 + k] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int o = tid + 256 * u;
            if (o < cnt * K) L[o] = bias ? lv[u] + Bs[o - (o / K) * K] : lv[u];
        }
    } else {
        for (int o = tid; o < cnt * K; o += 256) {
            const int img = o / K, k = o - img * K;
            float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // four chains: LDS latency overlaps
            for (int f = 0; f < F; f += 4) {
                a0 = fmaf(X(img, f), Wt(k, f), a0);
                a1 = fmaf(X(img, f + 1), Wt(k, f + 1), a1);
                a2 = fmaf(X(img, f + 2), Wt(k, f + 2), a2);
                a3 = fmaf(X(img, f + 3), Wt(k, f + 3), a3);
            }
            const float acc = (a0 + a1) + (a2 + a3);
            L[img * K + k] = bias ? acc + bias[z * b_cs + k] : acc;
        }
    }
    __syncthreads();
    // 2. cross-entropy (ce_kernel's operations and fp64 sum order)
    const float inv_n = cnt > 0 ? 1.0f / (float)cnt : 0.f;
    double lsum = 0.0;
    int corr = 0;
    if (K <= 16) {
        // a group of 16 lanes per image, the group's two images (g, g + 16; batch <= 32) side
        // by side so their shuffle chains overlap — each image's operations and order as before
        const int g = tid >> 4, l = tid & 15;
        float v[2], mx[2], se[2];
        int amax[2], tgt[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int img = g + 16 * u;  // < 32: L has 32 rows
            tgt[u] = img < cnt ? (SMALLK ? (int)Ts[img] : (int)targets[z * t_cs + img]) : 0;
            v[u] = l < K ? L[img * K + l] : -INFINITY;
            mx[u] = v[u];
            amax[u] = l < K ? l : K;
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float om = __shfl_xor(mx[u], o, 16);
                const int oa = __shfl_xor(amax[u], o, 16);
                if (om > mx[u] || (om == mx[u] && oa < amax[u])) { mx[u] = om; amax[u] = oa; }
            }
#pragma unroll
        for (int u = 0; u < 2; ++u) se[u] = l < K ? expf(v[u] - mx[u]) : 0.f;
#pragma unroll
        for (int o = 8; o > 0; o >>= 1)
#pragma unroll
            for (int u = 0; u < 2; ++u) se[u] += __shfl_xor(se[u], o, 16);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int img = g + 16 * u;
            if (img >= cnt) break;  // uniform over the group
            const float lse = logf(se[u]);
            if (l == 0) {
                li[img] = (double)(-((L[img * K + tgt[u]] - mx[u]) - lse));
                ci[img] = amax[u] == tgt[u];
            }
            if (l < K) {
                const float p = expf((v[u] - mx[u]) - lse);
                D[img * K + l] = (p - (l == tgt[u] ? 1.f : 0.f)) * inv_n;
            }
        }
        __syncthreads();
        if (tid < 4) {  // image order, the reads first
            double lv[8];
            int cv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                lv[j] = li[tid + 4 * j];
                cv[j] = ci[tid + 4 * j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (tid + 4 * j < cnt) {
                    lsum += lv[j];
                    corr += cv[j];
                }
            sl[tid] = lsum;
            sc[tid] = corr;
        }
    } else {
        for (int img = wid; img < cnt; img += 4) {
            const float* row = L + img * K;
            const int tgt = (int)targets[z * t_cs + img];
            float mx = -INFINITY;
            int amax = 0;
            for (int k = lane; k < K; k += 64) {
                const float v = row[k];
                if (v > mx) { mx = v; amax = k; }
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const float om = __shfl_xor(mx, o, 64);
                const int oa = __shfl_xor(amax, o, 64);
                if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
            }
            float se = 0.f;
            for (int k = lane; k < K; k += 64) se += expf(row[k] - mx);
            se = wave_sum(se);
            const float lse = logf(se);
            if (lane == 0) {
                lsum += (double)(-((row[tgt] - mx) - lse));
                corr += (amax == tgt);
            }
            for (int k = lane; k < K; k += 64) {
                const float p = expf((row[k] - mx) - lse);
                D[img * K + k] = (p - (k == tgt ? 1.f : 0.f)) * inv_n;
            }
        }
        if (lane == 0) {
            sl[wid] = lsum;
            sc[wid] = corr;
        }
    }
    __syncthreads();
    if (part == 0) {
        if (tid == 0) {
            const double tot = sl[0] + sl[1] + sl[2] + sl[3];
            const float batch_loss = cnt > 0 ? (float)(tot / (double)cnt) : 0.f;
            if (loss_out) loss_out[z] = batch_loss;
            if (acc_loss) acc_loss[z] = (rs0 ? 0.0 : al0) + (double)batch_loss;
            if (acc_correct) acc_correct[z] = (rs0 ? 0 : ac0) + sc[0] + sc[1] + sc[2] + sc[3];
            if (acc_seen) acc_seen[z] = (rs0 ? 0 : as0) + cnt;
        }
        for (int o = tid; o < cnt * K; o += 256) {
            logits[z * l_cs + o] = L[o];
            dlogits[z * d_cs + o] = D[o];
        }
        if (SMALLK && db && wid == 0) {  // four image groups per class, then xor-combined
            const int k = lane & 15, g = lane >> 4;
            float v = 0.f, dv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) dv[j] = D[(g + 4 * j) * K + k];  // < 32 x 16: in bounds
            if (k < K)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (g + 4 * j < cnt) v += dv[j];
            v += __shfl_xor(v, 16, 64);
            v += __shfl_xor(v, 32, 64);
            if (lane < K) db[z * db_cs + lane] = v;
        } else if (db && tid < K) {
            float v = 0.f;
            for (int b = 0; b < cnt; ++b) v += D[b * K + tid];
            db[z * db_cs + tid] = v;
        }
    }
    // 3. weight gradient, this block's share: dW[k][f] = sum_b D[b][k] x[b][f] (dw null: the
    // caller takes it elsewhere — DP-SGD clips it per image first)
    if (SMALLK && dw) {  // 16-column tiles of dW [K][F]; A = D^T (class x image), B = x
        const int mn = lane & 15, kk = lane >> 4;
        for (int tt = part + S * wid; tt < F / 16; tt += 4 * S) {
            const int f0 = tt * 16;
            float dr[8], xr2[8];  // operands read up front (in bounds: b < 32, mn < 16)
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int b = 4 * q + kk;
                const bool ok = b < cnt;
                const float dv = D[b * K + mn], xv = Xs[b * FP + f0 + mn];
                dr[q] = ok && mn < K ? dv : 0.f;
                xr2[q] = ok ? xv : 0.f;
            }
            hf32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (4 * q < cnt) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dr[q], xr2[q], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = 4 * kk + r;
                if (k < K) dw[z * dw_cs + (int64_t)k * F + f0 + mn] = acc[r];
            }
        }
    } else if (dw) {
        const int per = (K * F + S - 1) / S, e0 = part * per, e1 = min(K * F, e0 + per);
        for (int e = e0 + tid; e < e1; e += 256) {
            const int k = e / F, f = e - k * F;
            float a0 = 0.f, a1 = 0.f;
            int b = 0;
            for (; b + 1 < cnt; b += 2) {
                a0 = fmaf(D[b * K + k], X(b, f), a0);
                a1 = fmaf(D[(b + 1) * K + k], X(b + 1, f), a1);
            }
            if (b < cnt) a0 = fmaf(D[b * K + k], X(b, f), a0);
            dw[z * dw_cs + e] = a0 + a1;
        }
    }
    // 4. input gradient through Dropout + ReLU, this block's share: dx[b][f] = sum_k D[b][k] W[k][f]
    if (SMALLK && dx) {  // tiles of 16 images x 16 columns of dX; A = D (image x class), B = W
        const int mn = lane & 15, kk = lane >> 4;
        for (int tt = part + S * wid; tt < 2 * (F / 16); tt += 4 * S) {
            const int t = tt & 1, f0 = (tt >> 1) * 16;
            if (t * 16 >= cnt) continue;  // wave-uniform
            const int ia = t * 16 + mn;
            float dr[KMAX / 4], wr2[KMAX / 4];  // read up front (in bounds: ia < 32, k < 16)
#pragma unroll
            for (int q = 0; q < KMAX / 4; ++q) {
                const int k = 4 * q + kk;
                const float dv = D[ia * K + k], wv2 = Ws[k * FP + f0 + mn];
                dr[q] = k < K && ia < cnt ? dv : 0.f;
                wr2[q] = k < K ? wv2 : 0.f;
            }
            hf32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < KMAX / 4; ++q)
                if (4 * q < K) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dr[q], wr2[q], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int img = t * 16 + 4 * kk + r, f = f0 + mn;
                if (img < cnt) {
                    float v = acc[r];
                    if (mask) v = Ms[img * F + f] ? v * scale : 0.f;
                    if (relu_in && !(Xs[img * FP + f] > 0.f)) v = 0.f;
                    dx[z * dx_cs + (int64_t)img * F + f] = v;
                }
            }
        }
    } else if (dx) {
        const int e0 = dx_e0, e1 = dx_e1;
        for (int eb = e0 + tid; eb < e1; eb += 4 * 256) {  // keep-mask bytes of 4 outputs first
            uint8_t mk[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = eb + 256 * u;
                mk[u] = (mask && e < e1) ? mask[z * m_cs + e] : 1;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int e = eb + 256 * u;
                if (e >= e1) break;
                const int img = e / F, f = e - img * F;
                float acc = 0.f;
                for (int k = 0; k < K; ++k) acc = fmaf(D[img * K + k], Wt(k, f), acc);
                if (mask) acc = mk[u] ? acc * scale : 0.f;
                if (relu_in && !(X(img, f) > 0.f)) acc = 0.f;
                dx[z * dx_cs + e] = acc;
            }
        }
    }
}

// ------------------------------------------------------------------ evaluation metrics
// LocalTrainer.evaluate_model (training.py:307-360) / _validate_epoch (:214-242): per image
// the first-index argmax (torch.max) and the CE loss; per slot the fp64 loss sum and correct
// count (accumulated across launches, one block per slot: fixed order), per class the
// correct / total counts (integer atomics: order-independent, deterministic).
__global__ void __launch_bounds__(256)
eval_metrics_kernel(const float* __restrict__ logits, int64_t l_cs,
                    const int64_t* __restrict__ targets, int64_t t_cs,
                    const int32_t* __restrict__ counts, int batch, int K,
                    double* __restrict__ loss_sum, int64_t* __restrict__ correct,
                    unsigned long long* __restrict__ class_correct,
                    unsigned long long* __restrict__ class_total) {
    __shared__ double sl[4];
    __shared__ int sc[4];
    const int z = blockIdx.x;
    const int cnt = counts ? counts[z] : batch;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double lsum = 0.0;
    int corr = 0;
    for (int img = wid; img < cnt; img += 4) {
        const float* row = logits + z * l_cs + (int64_t)img * K;
        const int tgt = (int)targets[z * t_cs + img];
        float mx = -INFINITY;
        int amax = 0;
        for (int k = lane; k < K; k += 64) {
            const float v = row[k];
            if (v > mx) { mx = v; amax = k; }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float om = __shfl_xor(mx, o, 64);
            const int oa = __shfl_xor(amax, o, 64);
            if (om > mx || (om == mx && oa < amax)) { mx = om; amax = oa; }
        }
        float se = 0.f;
        for (int k = lane; k < K; k += 64) se += expf(row[k] - mx);
        se = wave_sum(se);
        if (lane == 0) {
            lsum += (double)(-((row[tgt] - mx) - logf(se)));
            const int hit = amax == tgt;
            corr += hit;
            if (class_total && tgt >= 0 && tgt < K) {
                atomicAdd(class_total + tgt, 1ull);
                if (hit) atomicAdd(class_correct + tgt, 1ull);
            }
        }
    }
    if (lane == 0) {
        sl[wid] = lsum;
        sc[wid] = corr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (loss_sum) loss_sum[z] += sl[0] + sl[1] + sl[2] + sl[3];
        if (correct) correct[z] += sc[0] + sc[1] + sc[2] + sc[3];
    }
}

// ------------------------------------------------------------------ global average pool
__global__ void __launch_bounds__(256)
avgpool_fwd_kernel(const float* __restrict__ x, int64_t x_cs, float* __restrict__ y, int64_t y_cs,
                   const int32_t* __restrict__ counts, int batch, int C, int HW) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int lane = threadIdx.x & 63;
    const int64_t planes = (int64_t)cnt * C;
    for (int64_t pl = blockIdx.x * 4 + (threadIdx.x >> 6); pl < planes; pl += gridDim.x * 4) {
        const float* b = x + z * x_cs + pl * HW;
        float s = 0.f;
        for (int p = lane; p < HW; p += 64) s += b[p];
        s = wave_sum(s);
        if (lane == 0) y[z * y_cs + pl] = s / (float)HW;
    }
}

__global__ void __launch_bounds__(256)
avgpool_bwd_kernel(const float* __restrict__ dy, int64_t dy_cs, float* __restrict__ dx,
                   int64_t dx_cs, const int32_t* __restrict__ counts, int batch, int C, int HW) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int64_t total = (int64_t)cnt * C * HW;
    const float inv = 1.0f / (float)HW;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x)
        dx[z * dx_cs + e] = dy[z * dy_cs + e / HW] * inv;
}

// ------------------------------------------------------------------ batch gather
// x[z][b][:] = data[idx[z*idx_cs + b]][:] ; y[z][b] = labels[idx[..]] for b < counts[z].
__global__ void __launch_bounds__(256)
gather_kernel(const float* __restrict__ data, const int64_t* __restrict__ labels,
              const int64_t* __restrict__ idx, int64_t idx_cs, float* __restrict__ x, int64_t x_cs,
              int64_t* __restrict__ y, int64_t y_cs, int64_t sample_elems,
              const int32_t* __restrict__ counts, int batch) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int64_t total = (int64_t)cnt * sample_elems;
    // four grid-stride elements per pass, loads ahead of stores (as gather_u8_kernel)
    constexpr int U = 4;
    const int64_t G = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e0 < total; e0 += U * G) {
        int64_t bq[U], oq[U], sq[U];
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = e0 + u * G;
            bq[u] = e < total ? e / sample_elems : 0;
            oq[u] = e - bq[u] * sample_elems;
            sq[u] = e < total ? idx[z * idx_cs + bq[u]] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = e0 + u * G < total ? data[sq[u] * sample_elems + oq[u]] : 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = e0 + u * G;
            if (e >= total) break;
            x[z * x_cs + e] = v[u];
            if (oq[u] == 0 && y) y[z * y_cs + bq[u]] = labels[sq[u]];
        }
    }
}

// ---- uint8 dataset -> normalised (and augmented) fp32 batch -----------------------
// torchvision's per-sample train transform of the reference's loaders
// (data_loader.py:298-301 MNIST: ToTensor + Normalize; :454-458 CIFAR: RandomCrop(32, 4)
// + RandomHorizontalFlip + ToTensor + Normalize), run on the chip over the raw uint8
// images (HWC, as torchvision datasets hold them) instead of on CPU loader workers:
//   v = (fl32(u8) / 255 - mean_c) / std_c         (to_tensor .div(255); normalize sub_, div_)
//   crop: padded(y + i, x + j) with zero padding (fill 0 before ToTensor);  flip after crop.
// Crop offsets / flip come from `aug_in` [S][B] uchar4 {i, j, flip, -} when given
// (replay), else from Philox(seed, (z, b)) and are then recorded to `aug_out` (nullable).
struct NormParams {
    float mean[4];
    float stdv[4];
};

__global__ void __launch_bounds__(256)
gather_u8_kernel(const uint8_t* __restrict__ data, const int64_t* __restrict__ labels,
                 const int64_t* __restrict__ idx, int64_t idx_cs, float* __restrict__ x,
                 int64_t x_cs, int64_t* __restrict__ y, int64_t y_cs,
                 const int32_t* __restrict__ counts, int batch, int C, int H, int W,
                 NormParams np, int pad, int flip, const uchar4* __restrict__ aug_in,
                 uchar4* __restrict__ aug_out, int64_t aug_cs, uint64_t seed_salt,
                 const uint64_t* __restrict__ seed_dev) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const uint32_t plane = (uint32_t)(H * W), per = plane * (uint32_t)C;
    const uint32_t total = (uint32_t)cnt * per;  // 32-bit index arithmetic (< 2^31 per client)
    const uint64_t seed = seed_salt + (seed_dev ? *seed_dev : 0ull);
    const uint64_t prow = philox_row(seed_dev, z);  // once, not per store
    // four grid-stride elements per pass, every load issued before the first store (r05: one
    // element per pass left two dependent round trips — sample index, then byte — per element).
    // Loads come in two waves (sample index and recorded augmentation, then the image byte and
    // the label), each from in-bounds addresses with the result selected after, so no load sits
    // under a branch with its use (r05: the byte load behind `in ?` and the recorded offsets
    // behind `if (aug_in)` had been one dependent round trip per element each)
    constexpr int U = 4;
    const uint32_t G = gridDim.x * blockDim.x;
    const bool aug = pad > 0 || flip;
    for (uint32_t e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += U * G) {
        uint32_t bq[U], rq[U];
        int cq[U], sy[U], sx[U];
        int64_t sq[U];
        uchar4 aq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * G;
            const uint32_t b = e < total ? e / per : 0u;
            bq[u] = b;
            rq[u] = e - b * per;
            sq[u] = idx[z * idx_cs + b];
            aq[u] = aug_in ? aug_in[z * aug_cs + b] : make_uchar4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * G, b = bq[u], r = rq[u];
            const int c = (int)(r / plane);
            const uint32_t p = r - (uint32_t)c * plane;
            const int yy = (int)(p / (uint32_t)W), xx = (int)(p - (uint32_t)yy * (uint32_t)W);
            int ci = pad, cj = pad, fl = 0;
            if (e < total && aug) {
                if (aug_in) {
                    ci = aq[u].x; cj = aq[u].y; fl = aq[u].z;
                } else {
                    const uint4 rr = Philox::gen(seed, prow, (uint64_t)b);
                    const uint32_t span = 2u * (uint32_t)pad + 1u;
                    ci = pad > 0 ? (int)(((uint64_t)rr.x * span) >> 32) : 0;
                    cj = pad > 0 ? (int)(((uint64_t)rr.y * span) >> 32) : 0;
                    fl = flip ? (int)(rr.z >> 31) : 0;
                    if (aug_out && r == 0) aug_out[z * aug_cs + b] = make_uchar4(ci, cj, fl, 0);
                }
            }
            const int sx0 = fl ? (W - 1 - xx) : xx;  // flip acts on the cropped image
            cq[u] = c;
            sy[u] = yy + ci - pad;
            sx[u] = sx0 + cj - pad;
        }
        uint32_t ub[U];
        int64_t lq[U];
        bool inq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            inq[u] = e0 + u * G < total && sy[u] >= 0 && sy[u] < H && sx[u] >= 0 && sx[u] < W;
            const int64_t off = inq[u] ? ((sq[u] * H + sy[u]) * W + sx[u]) * C + cq[u] : 0;
            ub[u] = data[off];
            lq[u] = labels[sq[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * G;
            if (e >= total) break;
            const float v = __fdiv_rn(inq[u] ? (float)ub[u] : 0.f, 255.f);
            x[z * x_cs + e] = __fdiv_rn(v - np.mean[cq[u]], np.stdv[cq[u]]);
            if (rq[u] == 0 && y) y[z * y_cs + bq[u]] = lq[u];
        }
    }
}

static int ew_grid(int64_t n) { return (int)std::min<int64_t>(std::max<int64_t>(ceil_div(n, 256), 1), 2048); }

}  // namespace fh

using namespace fh;

static int maxpool2_fwd_impl(const float* x, int64_t x_cs, const float* in_scale,
                             const float* in_shift, int64_t aff_cs, float* y, int64_t y_cs,
                             uint8_t* idx, int64_t i_cs, uint8_t* mask, int64_t m_cs,
                             const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                             int32_t H, int32_t W, int32_t drop_mode, float p_drop, uint64_t seed,
                             const uint64_t* seed_dev, void* stream, int32_t xh = 0,
                             int32_t xw = 0, int32_t yh = 0, int32_t yw = 0) {
    if (xh == 0) { xh = H; xw = W; yh = H / 2; yw = W / 2; }
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && H >= 2 && W >= 2, "maxpool2_fwd: bad shape");
    FH_REQUIRE(xh >= H && xw >= W && yh >= H / 2 && yw >= W / 2, "maxpool2_fwd: plane %dx%d / "
               "%dx%d smaller than the map %dx%d", xh, xw, yh, yw, H, W);
    FH_REQUIRE((H % 2) == 0 && (W % 2) == 0, "maxpool2_fwd: odd spatial size %dx%d", H, W);
    FH_REQUIRE(drop_mode >= 0 && drop_mode <= 2 && (drop_mode == 0 || mask), "maxpool2_fwd: mask");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "maxpool2_fwd: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && y && idx, "maxpool2_fwd: null pointer");
    const float keep = 1.0f - p_drop, scale = 1.0f / keep;
    const int64_t per = (int64_t)batch * C * (H / 2) * (W / 2);
    FH_LAUNCH(maxpool2_fwd_kernel, dim3(ew_grid(per), nclients), dim3(256), 0,
                       as_stream(stream), x, x_cs, y, y_cs, idx, i_cs, mask, m_cs, counts, batch, C,
                       H, W, drop_mode, keep, scale, seed, seed_dev, in_scale, in_shift, aff_cs,
                       xh, xw, yh, yw);
    FH_LAUNCH_CHECK("maxpool2_fwd");
    return FH_OK;
}

extern "C" int fh_maxpool2_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs, uint8_t* idx,
                               int64_t i_cs, uint8_t* mask, int64_t m_cs, const int32_t* counts,
                               int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                               int32_t drop_mode, float p_drop, uint64_t seed,
                               const uint64_t* seed_dev, void* stream) {
    return maxpool2_fwd_impl(x, x_cs, nullptr, nullptr, 0, y, y_cs, idx, i_cs, mask, m_cs, counts,
                             nclients, batch, C, H, W, drop_mode, p_drop, seed, seed_dev, stream);
}

extern "C" int fh_maxpool2_fwd_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                                      const float* in_shift, int64_t aff_cs, float* y,
                                      int64_t y_cs, uint8_t* idx, int64_t i_cs, uint8_t* mask,
                                      int64_t m_cs, const int32_t* counts, int32_t nclients,
                                      int32_t batch, int32_t C, int32_t H, int32_t W,
                                      int32_t drop_mode, float p_drop, uint64_t seed,
                                      const uint64_t* seed_dev, void* stream) {
    FH_REQUIRE(in_scale && in_shift, "maxpool2_fwd_bnrelu: null scale/shift");
    return maxpool2_fwd_impl(x, x_cs, in_scale, in_shift, aff_cs, y, y_cs, idx, i_cs, mask, m_cs,
                             counts, nclients, batch, C, H, W, drop_mode, p_drop, seed, seed_dev,
                             stream);
}

static int maxpool2_bwd_impl(const float* dy, int64_t dy_cs, const uint8_t* idx, int64_t i_cs,
                             const uint8_t* mask, int64_t m_cs, float p_drop, const float* xin,
                             int64_t x_cs, float* dx, int64_t dx_cs, const int32_t* counts,
                             int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                             void* stream, int32_t gh, int32_t gw, int32_t xh, int32_t xw,
                             const float* yin = nullptr, int64_t yin_cs = 0) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && H >= 2 && W >= 2 && !(H & 1) && !(W & 1),
               "maxpool2_bwd: bad shape");
    FH_REQUIRE(gh >= H / 2 && gw >= W / 2 && xh >= H && xw >= W, "maxpool2_bwd: plane %dx%d / "
               "%dx%d smaller than the map %dx%d", gh, gw, xh, xw, H, W);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && idx && dx, "maxpool2_bwd: null pointer");
    const float scale = 1.0f / (1.0f - p_drop);
    const int64_t per = (int64_t)batch * C * (H / 2) * (W / 2);
    FH_LAUNCH(maxpool2_bwd_kernel, dim3(ew_grid(per), nclients), dim3(256), 0,
                       as_stream(stream), dy, dy_cs, idx, i_cs, mask, m_cs, xin, x_cs, dx, dx_cs,
                       counts, batch, C, H, W, scale, gh, gw, xh, xw, yin, yin_cs);
    FH_LAUNCH_CHECK("maxpool2_bwd");
    return FH_OK;
}

extern "C" int fh_maxpool2_bwd(const float* dy, int64_t dy_cs, const uint8_t* idx, int64_t i_cs,
                               const uint8_t* mask, int64_t m_cs, float p_drop, const float* xin,
                               int64_t x_cs, float* dx, int64_t dx_cs, const int32_t* counts,
                               int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                               void* stream) {
    return maxpool2_bwd_impl(dy, dy_cs, idx, i_cs, mask, m_cs, p_drop, xin, x_cs, dx, dx_cs,
                             counts, nclients, batch, C, H, W, stream, H / 2, W / 2, H, W);
}

// The same max-pools on maps embedded in larger planes (top-left corner; the direct-conv
// path runs SimpleCNN's 14x14 conv on 16x16 planes with a zero ring): fwd x planes
// xh x xw, y planes yh x yw; bwd dy planes gh x gw, dx / xin planes xh x xw.  The pool
// never writes outside the map, so a zero ring stays zero.
extern "C" int fh_maxpool2_fwd_pitched(const float* x, int64_t x_cs, float* y, int64_t y_cs,
                                       uint8_t* idx, int64_t i_cs, uint8_t* mask, int64_t m_cs,
                                       const int32_t* counts, int32_t nclients, int32_t batch,
                                       int32_t C, int32_t H, int32_t W, int32_t drop_mode,
                                       float p_drop, uint64_t seed, const uint64_t* seed_dev,
                                       int32_t xh, int32_t xw, int32_t yh, int32_t yw,
                                       void* stream) {
    FH_REQUIRE(xh > 0 && xw > 0 && yh > 0 && yw > 0, "maxpool2_fwd_pitched: bad planes");
    return maxpool2_fwd_impl(x, x_cs, nullptr, nullptr, 0, y, y_cs, idx, i_cs, mask, m_cs, counts,
                             nclients, batch, C, H, W, drop_mode, p_drop, seed, seed_dev, stream,
                             xh, xw, yh, yw);
}

extern "C" int fh_maxpool2_bwd_pitched(const float* dy, int64_t dy_cs, const uint8_t* idx,
                                       int64_t i_cs, const uint8_t* mask, int64_t m_cs,
                                       float p_drop, const float* xin, int64_t x_cs, float* dx,
                                       int64_t dx_cs, const int32_t* counts, int32_t nclients,
                                       int32_t batch, int32_t C, int32_t H, int32_t W, int32_t gh,
                                       int32_t gw, int32_t xh, int32_t xw, void* stream) {
    return maxpool2_bwd_impl(dy, dy_cs, idx, i_cs, mask, m_cs, p_drop, xin, x_cs, dx, dx_cs,
                             counts, nclients, batch, C, H, W, stream, gh, gw, xh, xw);
}

// fh_maxpool2_bwd_pitched with the ReLU mask taken from the pooled output y (planes gh x gw)
// instead of the full-resolution ReLU output (after fh_conv2d_c1_pool_fwd, which never wrote it)
extern "C" int fh_maxpool2_bwd_ymask(const float* dy, int64_t dy_cs, const uint8_t* idx,
                                     int64_t i_cs, const float* y, int64_t y_cs, float* dx,
                                     int64_t dx_cs, const int32_t* counts, int32_t nclients,
                                     int32_t batch, int32_t C, int32_t H, int32_t W, int32_t gh,
                                     int32_t gw, int32_t xh, int32_t xw, void* stream) {
    FH_REQUIRE(y || nclients == 0, "maxpool2_bwd_ymask: null pooled output");
    return maxpool2_bwd_impl(dy, dy_cs, idx, i_cs, nullptr, 0, 0.f, nullptr, 0, dx, dx_cs, counts,
                             nclients, batch, C, H, W, stream, gh, gw, xh, xw, y, y_cs);
}

extern "C" int fh_dropout_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs, uint8_t* mask,
                              int64_t m_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                              int64_t per_img, int32_t drop_mode, float p_drop, uint64_t seed,
                              const uint64_t* seed_dev, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && per_img > 0, "dropout_fwd: bad shape");
    FH_REQUIRE((drop_mode == 1 || drop_mode == 2) && mask, "dropout_fwd: mask mode");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "dropout_fwd: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && y, "dropout_fwd: null pointer");
    const float keep = 1.0f - p_drop, scale = 1.0f / keep;
    FH_LAUNCH(dropout_fwd_kernel, dim3(ew_grid(batch * per_img), nclients), dim3(256), 0,
                       as_stream(stream), x, x_cs, y, y_cs, mask, m_cs, counts, batch, per_img,
                       drop_mode, keep, scale, seed, seed_dev);
    FH_LAUNCH_CHECK("dropout_fwd");
    return FH_OK;
}

extern "C" int fh_dropout_bwd(const float* dy, int64_t dy_cs, const uint8_t* mask, int64_t m_cs,
                              float p_drop, const float* relu_out, int64_t r_cs, float* dx,
                              int64_t dx_cs, const int32_t* counts, int32_t nclients,
                              int32_t batch, int64_t per_img, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && per_img > 0, "dropout_bwd: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && dx, "dropout_bwd: null pointer");
    const float scale = 1.0f / (1.0f - p_drop);
    FH_LAUNCH(dropout_bwd_kernel, dim3(ew_grid(batch * per_img), nclients), dim3(256), 0,
                       as_stream(stream), dy, dy_cs, mask, m_cs, relu_out, r_cs, dx, dx_cs, counts,
                       batch, per_img, scale);
    FH_LAUNCH_CHECK("dropout_bwd");
    return FH_OK;
}

extern "C" int fh_ce_fwd_bwd(const float* logits, int64_t l_cs, const int64_t* targets,
                             int64_t t_cs, float* dlogits, int64_t d_cs, float* loss_out,
                             double* acc_loss, int64_t* acc_correct, int64_t* acc_seen,
                             const int32_t* reset, const int32_t* counts, int32_t nclients,
                             int32_t batch, int32_t num_classes, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && num_classes > 0, "ce_fwd_bwd: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(logits && targets && dlogits, "ce_fwd_bwd: null pointer");
    FH_LAUNCH(ce_kernel, dim3(nclients), dim3(256), 0, as_stream(stream), logits, l_cs,
                       targets, t_cs, dlogits, d_cs, loss_out, acc_loss, acc_correct, acc_seen,
                       reset, counts, batch, num_classes);
    FH_LAUNCH_CHECK("ce_fwd_bwd");
    return FH_OK;
}

extern "C" int fh_linear_head_ce(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                                 const float* bias, int64_t b_cs, const int64_t* targets,
                                 int64_t t_cs, float* logits, int64_t l_cs, float* dlogits,
                                 int64_t d_cs, float* loss_out, double* acc_loss,
                                 int64_t* acc_correct, int64_t* acc_seen, const int32_t* reset,
                                 float* dw, int64_t dw_cs, float* db, int64_t db_cs, float* dx,
                                 int64_t dx_cs, const uint8_t* mask, int64_t m_cs, float p_drop,
                                 int32_t relu_in, const int32_t* counts, int32_t nclients,
                                 int32_t batch, int32_t in_f, int32_t num_classes, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && in_f > 0 && num_classes > 0, "linear_head_ce: bad shape");
    FH_REQUIRE(batch <= 32 && num_classes <= 128 && in_f % 4 == 0, "linear_head_ce: needs batch "
               "<= 32, <= 128 classes and in_f %% 4 == 0 (got %d, %d, %d)", batch, num_classes,
               in_f);
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "linear_head_ce: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && w && targets && logits && dlogits && (dw || !db),
               "linear_head_ce: null pointer");
    const dim3 grid(kHeadBlocks, nclients);
    const float scale = 1.0f / (1.0f - p_drop);
    if (num_classes <= 16 && in_f <= 256 && in_f % 16 == 0)
        FH_LAUNCH(linear_head_ce_kernel<true>, grid, dim3(256), 0, as_stream(stream), x, x_cs, w,
                  w_cs, bias, b_cs, targets, t_cs, logits, l_cs, dlogits, d_cs, loss_out,
                  acc_loss, acc_correct, acc_seen, reset, dw, dw_cs, db, db_cs, dx, dx_cs, mask,
                  m_cs, scale, relu_in, counts, batch, in_f, num_classes);
    else
        FH_LAUNCH(linear_head_ce_kernel<false>, grid, dim3(256), 0, as_stream(stream), x, x_cs, w,
                  w_cs, bias, b_cs, targets, t_cs, logits, l_cs, dlogits, d_cs, loss_out,
                  acc_loss, acc_correct, acc_seen, reset, dw, dw_cs, db, db_cs, dx, dx_cs, mask,
                  m_cs, scale, relu_in, counts, batch, in_f, num_classes);
    FH_LAUNCH_CHECK("linear_head_ce");
    return FH_OK;
}

extern "C" int fh_eval_metrics(const float* logits, int64_t l_cs, const int64_t* targets,
                               int64_t t_cs, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t num_classes, double* loss_sum,
                               int64_t* correct, int64_t* class_correct, int64_t* class_total,
                               void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && num_classes > 0, "eval_metrics: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(logits && targets, "eval_metrics: null pointer");
    FH_REQUIRE((class_correct == nullptr) == (class_total == nullptr),
               "eval_metrics: class_correct and class_total go together");
    FH_LAUNCH(eval_metrics_kernel, dim3(nclients), dim3(256), 0, as_stream(stream),
                       logits, l_cs, targets, t_cs, counts, batch, num_classes, loss_sum, correct,
                       reinterpret_cast<unsigned long long*>(class_correct),
                       reinterpret_cast<unsigned long long*>(class_total));
    FH_LAUNCH_CHECK("eval_metrics");
    return FH_OK;
}

extern "C" int fh_avgpool_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs,
                              const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                              int32_t HW, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "avgpool_fwd: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && y, "avgpool_fwd: null pointer");
    const int64_t planes = (int64_t)batch * C;
    FH_LAUNCH(avgpool_fwd_kernel, dim3(ew_grid(planes * 64), nclients), dim3(256), 0,
                       as_stream(stream), x, x_cs, y, y_cs, counts, batch, C, HW);
    FH_LAUNCH_CHECK("avgpool_fwd");
    return FH_OK;
}

extern "C" int fh_avgpool_bwd(const float* dy, int64_t dy_cs, float* dx, int64_t dx_cs,
                              const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                              int32_t HW, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "avgpool_bwd: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(dy && dx, "avgpool_bwd: null pointer");
    FH_LAUNCH(avgpool_bwd_kernel, dim3(ew_grid((int64_t)batch * C * HW), nclients),
                       dim3(256), 0, as_stream(stream), dy, dy_cs, dx, dx_cs, counts, batch, C, HW);
    FH_LAUNCH_CHECK("avgpool_bwd");
    return FH_OK;
}

extern "C" int fh_gather_batch(const float* data, const int64_t* labels, const int64_t* idx,
                               int64_t idx_cs, float* x, int64_t x_cs, int64_t* y, int64_t y_cs,
                               int64_t sample_elems, const int32_t* counts, int32_t nclients,
                               int32_t batch, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && sample_elems > 0, "gather_batch: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(data && idx && x && (!y || labels), "gather_batch: null pointer");
    FH_LAUNCH(gather_kernel, dim3(ew_grid(batch * sample_elems), nclients), dim3(256), 0,
                       as_stream(stream), data, labels, idx, idx_cs, x, x_cs, y, y_cs, sample_elems,
                       counts, batch);
    FH_LAUNCH_CHECK("gather_batch");
    return FH_OK;
}

extern "C" int fh_gather_u8(const uint8_t* data, const int64_t* labels, const int64_t* idx,
                            int64_t idx_cs, float* x, int64_t x_cs, int64_t* y, int64_t y_cs,
                            const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                            int32_t H, int32_t W, const float* mean, const float* stdv,
                            int32_t pad, int32_t flip, const uint8_t* aug_in, uint8_t* aug_out,
                            int64_t aug_cs, uint64_t seed, const uint64_t* seed_dev,
                            void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C >= 1 && C <= 4 && H > 0 && W > 0,
               "gather_u8: bad shape (C must be 1..4)");
    FH_REQUIRE(pad >= 0 && pad <= 127, "gather_u8: pad out of range");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(data && idx && x && (!y || labels) && mean && stdv, "gather_u8: null pointer");
    NormParams np;
    for (int c = 0; c < 4; ++c) {
        np.mean[c] = c < C ? mean[c] : 0.f;
        np.stdv[c] = c < C ? stdv[c] : 1.f;
    }
    FH_LAUNCH(gather_u8_kernel, dim3(ew_grid((int64_t)batch * C * H * W), nclients),
                       dim3(256), 0, as_stream(stream), data, labels, idx, idx_cs, x, x_cs, y, y_cs,
                       counts, batch, C, H, W, np, pad, flip,
                       reinterpret_cast<const uchar4*>(aug_in), reinterpret_cast<uchar4*>(aug_out),
                       aug_cs, seed, seed_dev);
    FH_LAUNCH_CHECK("gather_u8");
    return FH_OK;
}
