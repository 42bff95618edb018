// bn.hip — BatchNorm2d for client-packed activations (train fwd / eval fwd / bwd).
//
// Reference: nn.BatchNorm2d in CIFAR10CNN and FederatedResNet
// (src/shared/models_pytorch.py:108-120, 176-187), train-mode statistics over
// the valid images of each client, momentum 0.1, eps 1e-5, unbiased running
// variance — ATen CPU accumulates these in double (acc_type<float>); so do we.
//
// Each (client, channel) reduction is split over S blocks ("slices" of the
// channel's cnt*HW elements) so that even one client fills the chip; the S
// partials go to a caller workspace and are merged in a fixed order by the
// second kernel (deterministic).  Element loops are float4 when HW % 4 == 0.
//   train fwd : stats  (read x)            -> partial (sum x, sum x^2) in fp64
//               apply  (read x [,res], write y = relu?(x*alpha + beta [+res]))
//   bwd       : reduce (read dy, y, x [, write dres])  -> partial (sum g, sum (x-mean) g)
//               apply  (read dy, y, x, write dx = ((g - mean g) - (x-mean) k) invstd w)
// Fused: the ReLU that follows BN (forward) and its mask (backward, g = dy*(y>0)),
// and the ResNet residual add (forward) / residual-branch gradient (backward).
#include "fh_common.h"
#include "splitbn.h"

namespace fh {

struct BNArgs {
    const float* x;
    float* y;
    const float* res;
    const float* dy;
    const float* yout;
    float* dx;
    float* dres;
    const float* gamma;
    const float* beta;
    float* rmean;
    float* rvar;
    float* save_mean;
    float* save_invstd;
    float* dgamma;
    float* dbeta;
    double* part;  // [z][C][SP][2]
    int SP;        // partial pairs per (client, channel) merge() adds (S, or conv tiles)
    int64_t x_cs, y_cs, res_cs, dy_cs, yo_cs, dx_cs, dres_cs, p_cs, r_cs, g_cs;
    const int32_t* counts;
    int batch, C, HW, S, chunk;  // chunk: elements per slice (multiple of 4)
    float eps, momentum;
    int relu;
    int vec;  // float4 element path (HW % 4 == 0; pooled input also needs W % 4 == 0)
    FastDiv fd_hw;
    // backward through a 2x2 max-pool (+dropout): dy is not materialised; the gradient
    // of element (img,c,y,x) is dpool[img,c,y/2,x/2] (x dropout keep/scale) routed by
    // the window argmax pidx (== (y&1)*2 + (x&1)), else 0
    const float* dpool;
    const uint8_t* pidx;
    const uint8_t* pmask;
    int64_t dp_cs, pi_cs, pm_cs;
    float pscale;
    int W;
    FastDiv fd_w;
};

// Visit this block's slice of channel c of client z: f(offset_within_client_tensor, nvec)
// nvec = 4 (float4 at offset) or 1 (scalar).
template <class F>
__device__ __forceinline__ void for_slice(const BNArgs& a, int z, int c, int s, F&& f) {
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int n = cnt * a.HW;
    const int e0 = s * a.chunk, e1 = min(n, e0 + a.chunk);
    const int64_t istride = (int64_t)a.C * a.HW, coff = (int64_t)c * a.HW;
    if (a.vec) {
        for (int e = e0 + threadIdx.x * 4; e < e1; e += 256 * 4) {
            uint32_t img, p;
            a.fd_hw.divmod(e, img, p);
            f(img * istride + coff + p, 4);
        }
    } else {
        for (int e = e0 + threadIdx.x; e < e1; e += 256) {
            uint32_t img, p;
            a.fd_hw.divmod(e, img, p);
            f(img * istride + coff + p, 1);
        }
    }
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// Merge channel c's S partials -> (sum0, sum1), wave-cooperative: lane l adds partials
// l, l+64, ... in order, then an xor-shuffle tree; a fixed order, the same result in every
// lane.  Every lane of the calling wave must call it with the same (z, c).  (A sequential
// merge by one thread was S/8 dependent L2 round trips: the finalize on the critical path.)
__device__ __forceinline__ void merge(const BNArgs& a, int z, int c, double& s0, double& s1) {
    const double2* p = reinterpret_cast<const double2*>(a.part + (((int64_t)z * a.C + c) * a.SP) * 2);
    s0 = 0.0;
    s1 = 0.0;
    for (int i = threadIdx.x & 63; i < a.SP; i += 64) {
        const double2 v = p[i];
        s0 += v.x;
        s1 += v.y;
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
}

__global__ void __launch_bounds__(256) bn_stats_kernel(const BNArgs a) {
    __shared__ double red[4];
    const int s = blockIdx.x, c = blockIdx.y, z = blockIdx.z;
    const float* xz = a.x + z * a.x_cs;
    double s0 = 0.0, s1 = 0.0;
    for_slice(a, z, c, s, [&](int64_t o, int nv) {
        if (nv == 4) {
            const float4 v = ld4(xz + o);
            s0 += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
            s1 += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
        } else {
            const double v = xz[o];
            s0 += v;
            s1 += v * v;
        }
    });
    s0 = block_sum_256(s0, red);
    s1 = block_sum_256(s1, red);
    if (threadIdx.x == 0) {
        double* p = a.part + ((((int64_t)z * a.C + c) * a.S) + s) * 2;
        p[0] = s0;
        p[1] = s1;
    }
}

__global__ void __launch_bounds__(256) bn_apply_kernel(const BNArgs a) {
    const int s = blockIdx.x, c = blockIdx.y, z = blockIdx.z;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int64_t n = (int64_t)cnt * a.HW;
    double sum, sq;
    merge(a, z, c, sum, sq);
    const double mean = n > 0 ? sum / (double)n : 0.0;
    double var = n > 0 ? sq / (double)n - mean * mean : 0.0;
    if (var < 0.0) var = 0.0;
    const double invstd = n > 0 ? 1.0 / sqrt(var + (double)a.eps) : 0.0;
    const float meanf = (float)mean, invstdf = (float)invstd;
    if (s == 0 && threadIdx.x == 0) {
        a.save_mean[z * a.C + c] = meanf;
        a.save_invstd[z * a.C + c] = invstdf;
        if (a.rmean && n > 0) {
            const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
            float* rm = a.rmean + z * a.r_cs + c;
            float* rv = a.rvar + z * a.r_cs + c;
            *rm = (float)((double)a.momentum * mean + (1.0 - (double)a.momentum) * (double)*rm);
            *rv = (float)((double)a.momentum * unb + (1.0 - (double)a.momentum) * (double)*rv);
        }
    }
    // y = x*alpha + beta'  (alpha = invstd*w, beta' = b - mean*alpha), [+res], [relu]
    const float alpha = invstdf * a.gamma[z * a.p_cs + c];
    const float bconst = a.beta[z * a.p_cs + c] - meanf * alpha;
    const float* xz = a.x + z * a.x_cs;
    float* yz = a.y + z * a.y_cs;
    const float* rz = a.res ? a.res + z * a.res_cs : nullptr;
    const int relu = a.relu;
    for_slice(a, z, c, s, [&](int64_t o, int nv) {
        if (nv == 4) {
            float4 v = ld4(xz + o);
            v.x = v.x * alpha + bconst;
            v.y = v.y * alpha + bconst;
            v.z = v.z * alpha + bconst;
            v.w = v.w * alpha + bconst;
            if (rz) {
                const float4 r = ld4(rz + o);
                v.x = v.x + r.x; v.y = v.y + r.y; v.z = v.z + r.z; v.w = v.w + r.w;
            }
            if (relu) {
                v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f);
                v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
            }
            st4(yz + o, v);
        } else {
            float v = xz[o] * alpha + bconst;
            if (rz) v = v + rz[o];
            if (relu) v = fmaxf(v, 0.f);
            yz[o] = v;
        }
    });
}

// Train-mode statistics without the apply pass: per (client, channel) the merged moments
// become save_mean / save_invstd, the running-stat update, and the affine the consumer
// applies on load (scale = invstd*w, shift = b - mean*scale: bn_apply_kernel's alpha and
// beta', same operations, so relu(x*scale + shift) is bit-identical to its output).
__global__ void __launch_bounds__(256) bn_finalize_kernel(const BNArgs a, float* scale,
                                                          float* shift, int64_t s_cs) {
    // one wave per channel (merge() is wave-cooperative)
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6), z = blockIdx.y;
    if (c >= a.C) return;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int64_t n = (int64_t)cnt * a.HW;
    double sum, sq;
    merge(a, z, c, sum, sq);
    if ((threadIdx.x & 63) != 0) return;
    const double mean = n > 0 ? sum / (double)n : 0.0;
    double var = n > 0 ? sq / (double)n - mean * mean : 0.0;
    if (var < 0.0) var = 0.0;
    const double invstd = n > 0 ? 1.0 / sqrt(var + (double)a.eps) : 0.0;
    const float meanf = (float)mean, invstdf = (float)invstd;
    a.save_mean[z * a.C + c] = meanf;
    a.save_invstd[z * a.C + c] = invstdf;
    if (a.rmean && n > 0) {
        const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
        float* rm = a.rmean + z * a.r_cs + c;
        float* rv = a.rvar + z * a.r_cs + c;
        *rm = (float)((double)a.momentum * mean + (1.0 - (double)a.momentum) * (double)*rm);
        *rv = (float)((double)a.momentum * unb + (1.0 - (double)a.momentum) * (double)*rv);
    }
    const float alpha = invstdf * a.gamma[z * a.p_cs + c];
    const float bconst = a.beta[z * a.p_cs + c] - meanf * alpha;
    scale[z * s_cs + c] = alpha;
    shift[z * s_cs + c] = bconst;
}

// BatchNorm finalize fused into the 2x2 max-pool (+dropout) that consumes the BN-ReLU output
// (CIFAR10CNN bn2/bn4/bn6 -> relu -> pool -> dropout, models_pytorch.py:139-155): one launch
// instead of fh_bn_finalize_tiles + fh_maxpool2_fwd_bnrelu.  Blocks own one channel of one
// client (BPC blocks per channel split its pooled elements); each merges the channel's
// per-tile partials from the producing conv's epilogue (lane-strided fp64 sums combined by
// xor-shuffles: a fixed order, the same in every block of the channel), derives the affine
// with bn_finalize_kernel's operations, and pools relu(x*alpha + beta') exactly as
// maxpool2_fwd_kernel (window argmax, Philox keep-mask keyed by the pooled element index).
// Block 0 of the channel writes save_mean / save_invstd, the running statistics and the
// affine.
constexpr int kPoolEpt = 4;  // pooled elements per thread in maxpool2_bnfin_kernel

__global__ void __launch_bounds__(256)
maxpool2_bnfin_kernel(const BNArgs a, float* __restrict__ scale_out, float* __restrict__ shift_out,
                      int64_t s_cs, const float* __restrict__ x, int64_t x_cs,
                      float* __restrict__ y, int64_t y_cs, uint8_t* __restrict__ idx, int64_t i_cs,
                      uint8_t* __restrict__ mask, int64_t m_cs, int H, int W, int drop_mode,
                      float keep_prob, float dscale, uint64_t seed_salt,
                      const uint64_t* __restrict__ seed_dev, int bpc) {
    __shared__ float s_aff[2];
    const int z = blockIdx.y, c = blockIdx.x / bpc, sb = blockIdx.x - c * bpc;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int64_t n = (int64_t)cnt * a.HW;
    // this thread's windows (kPoolEpt pooled elements, 256 apart: host
    // bpc = ceil(batch*ohw / (256*kPoolEpt))), loaded before the merge so the loads are in
    // flight across it and one merge serves kPoolEpt*256 elements
    const int OH = H / 2, OW = W / 2, ohw = OH * OW;
    const int64_t per_ch = (int64_t)cnt * ohw;
    int64_t e[kPoolEpt];
    float xv[kPoolEpt][4];
#pragma unroll
    for (int k = 0; k < kPoolEpt; ++k) {
        const int64_t q = ((int64_t)sb * kPoolEpt + k) * 256 + threadIdx.x;
        e[k] = -1;
        xv[k][0] = xv[k][1] = xv[k][2] = xv[k][3] = 0.f;
        if (q < per_ch) {
            const int img = (int)(q / ohw), r = (int)(q - (int64_t)img * ohw);
            const int oh = r / OW, ow = r - oh * OW;
            const int64_t plane = (int64_t)img * a.C + c;
            e[k] = plane * ohw + r;  // maxpool2_fwd_kernel's element index
            const float* pp = x + z * x_cs + plane * H * W + (2 * oh) * W + 2 * ow;
            xv[k][0] = pp[0]; xv[k][1] = pp[1]; xv[k][2] = pp[W]; xv[k][3] = pp[W + 1];
        }
    }
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        double s0, s1;
        merge(a, z, c, s0, s1);
        if (lane == 0) {
            const double mean = n > 0 ? s0 / (double)n : 0.0;
            double var = n > 0 ? s1 / (double)n - mean * mean : 0.0;
            if (var < 0.0) var = 0.0;
            const double invstd = n > 0 ? 1.0 / sqrt(var + (double)a.eps) : 0.0;
            const float meanf = (float)mean, invstdf = (float)invstd;
            const float alpha = invstdf * a.gamma[z * a.p_cs + c];
            const float bconst = a.beta[z * a.p_cs + c] - meanf * alpha;
            s_aff[0] = alpha;
            s_aff[1] = bconst;
            if (sb == 0) {
                a.save_mean[z * a.C + c] = meanf;
                a.save_invstd[z * a.C + c] = invstdf;
                if (a.rmean && n > 0) {
                    const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
                    float* rm = a.rmean + z * a.r_cs + c;
                    float* rv = a.rvar + z * a.r_cs + c;
                    *rm = (float)((double)a.momentum * mean + (1.0 - (double)a.momentum) * (double)*rm);
                    *rv = (float)((double)a.momentum * unb + (1.0 - (double)a.momentum) * (double)*rv);
                }
                scale_out[z * s_cs + c] = alpha;
                shift_out[z * s_cs + c] = bconst;
            }
        }
    }
    __syncthreads();
    const float s = s_aff[0], t = s_aff[1];
    const uint64_t seed = seed_salt + (seed_dev ? *seed_dev : 0ull);
    const uint64_t prow = drop_mode == 1 ? philox_row(seed_dev, z) : 0ull;  // once, not per store
#pragma unroll
    for (int k = 0; k < kPoolEpt; ++k) {
        if (e[k] < 0) continue;
        const float v0 = fmaxf(xv[k][0] * s + t, 0.f), v1 = fmaxf(xv[k][1] * s + t, 0.f);
        const float v2 = fmaxf(xv[k][2] * s + t, 0.f), v3 = fmaxf(xv[k][3] * s + t, 0.f);
        float m = v0;
        int am = 0;
        if (v1 > m) { m = v1; am = 1; }
        if (v2 > m) { m = v2; am = 2; }
        if (v3 > m) { m = v3; am = 3; }
        idx[z * i_cs + e[k]] = (uint8_t)am;
        if (drop_mode) {
            uint8_t keep;
            if (drop_mode == 1) {
                const uint4 rr = Philox::gen(seed, prow, (uint64_t)e[k]);
                keep = u01(rr.x) <= keep_prob ? 1 : 0;
                mask[z * m_cs + e[k]] = keep;
            } else {
                keep = mask[z * m_cs + e[k]];
            }
            m = keep ? m * dscale : 0.f;
        }
        y[z * y_cs + e[k]] = m;
    }
}

// eval mode: running statistics (LocalTrainer._validate_epoch / evaluate_model)
__global__ void __launch_bounds__(256) bn_eval_kernel(const BNArgs a) {
    const int s = blockIdx.x, c = blockIdx.y, z = blockIdx.z;
    const float invstd = (float)(1.0 / sqrt((double)a.rvar[z * a.r_cs + c] + (double)a.eps));
    const float alpha = invstd * a.gamma[z * a.p_cs + c];
    const float bconst = a.beta[z * a.p_cs + c] - a.rmean[z * a.r_cs + c] * alpha;
    const float* xz = a.x + z * a.x_cs;
    float* yz = a.y + z * a.y_cs;
    const float* rz = a.res ? a.res + z * a.res_cs : nullptr;
    for_slice(a, z, c, s, [&](int64_t o, int nv) {
        for (int q = 0; q < nv; ++q) {
            float v = xz[o + q] * alpha + bconst;
            if (rz) v = v + rz[o + q];
            if (a.relu) v = fmaxf(v, 0.f);
            yz[o + q] = v;
        }
    });
}


// upstream gradient at client-tensor offset o (before the ReLU mask): dy[o], or routed
// from the pooled gradient (maxpool2_bwd semantics, layers.hip)
__device__ __forceinline__ float pooled_g(const BNArgs& a, int z, int64_t o) {
    uint32_t y, x;
    const int64_t plane = o / a.HW;  // img*C + c
    a.fd_w.divmod((uint32_t)(o - plane * a.HW), y, x);
    const int64_t e = plane * (a.HW >> 2) + (int64_t)(y >> 1) * (a.W >> 1) + (x >> 1);
    if (a.pidx[z * a.pi_cs + e] != (int)(((y & 1) << 1) | (x & 1))) return 0.f;
    float g = a.dpool[z * a.dp_cs + e];
    if (a.pmask) g = a.pmask[z * a.pm_cs + e] ? g * a.pscale : 0.f;
    return g;
}

__device__ __forceinline__ float4 upstream4(const BNArgs& a, int z, int64_t o) {
    if (!a.dpool) return ld4(a.dy + z * a.dy_cs + o);
    // 4 consecutive columns (x % 4 == 0) = 2 pooled windows of one pooled row
    uint32_t y, x;
    const int64_t plane = o / a.HW;
    a.fd_w.divmod((uint32_t)(o - plane * a.HW), y, x);
    const int64_t e = plane * (a.HW >> 2) + (int64_t)(y >> 1) * (a.W >> 1) + (x >> 1);
    const int r = (y & 1) << 1;
    // every load unconditional (a null keep-mask reads the argmax bytes) and each keep byte
    // folded into its argmax code, which every result uses: r05 — under `if (pmask)` each mask
    // byte's load and use sat in a branch of their own, a dependent round trip per byte
    const uint8_t* pk = a.pmask ? a.pmask + z * a.pm_cs : a.pidx + z * a.pi_cs;
    float g0 = a.dpool[z * a.dp_cs + e], g1 = a.dpool[z * a.dp_cs + e + 1];
    const int c0 = a.pidx[z * a.pi_cs + e] | (pk[e] ? 4 : 0);
    const int c1 = a.pidx[z * a.pi_cs + e + 1] | (pk[e + 1] ? 4 : 0);
    const bool dm = a.pmask != nullptr;
    const float h0 = dm ? g0 * a.pscale : g0, h1 = dm ? g1 * a.pscale : g1;
    g0 = (!dm || (c0 & 4)) ? h0 : 0.f;
    g1 = (!dm || (c1 & 4)) ? h1 : 0.f;
    const int i0 = c0 & 3, i1 = c1 & 3;
    return make_float4(i0 == r ? g0 : 0.f, i0 == (r | 1) ? g0 : 0.f, i1 == r ? g1 : 0.f,
                       i1 == (r | 1) ? g1 : 0.f);
}

__device__ __forceinline__ float upstream1(const BNArgs& a, int z, int64_t o) {
    return a.dpool ? pooled_g(a, z, o) : a.dy[z * a.dy_cs + o];
}

// ReLU mask of the backward: from the stored forward output (yout > 0), or — no residual
// add in between — recomputed from x exactly as the forward evaluated it
// (x*alpha + beta' > 0 with the same fp32 operations), which saves reading yout.
struct ReluMask {
    int mode;  // 0 none, 1 yout, 2 recompute
    const float* yo;
    float alpha, bconst;
    __device__ ReluMask(const BNArgs& a, int z, int c, float mean, float invstd) {
        mode = !a.relu ? 0 : (a.yout ? 1 : 2);
        yo = mode == 1 ? a.yout + z * a.yo_cs : nullptr;
        alpha = 0.f;
        bconst = 0.f;
        if (mode == 2) {
            alpha = invstd * a.gamma[z * a.p_cs + c];
            bconst = a.beta[z * a.p_cs + c] - mean * alpha;
        }
    }
    __device__ __forceinline__ bool keep(float x, int64_t o) const {
        if (mode == 0) return true;
        if (mode == 1) return yo[o] > 0.f;
        return x * alpha + bconst > 0.f;
    }
    __device__ __forceinline__ float4 apply4(float4 g, float4 xv, int64_t o) const {
        if (mode == 0) return g;
        float4 m;
        if (mode == 1) {
            m = ld4(yo + o);
        } else {
            m.x = xv.x * alpha + bconst; m.y = xv.y * alpha + bconst;
            m.z = xv.z * alpha + bconst; m.w = xv.w * alpha + bconst;
        }
        g.x = m.x > 0.f ? g.x : 0.f; g.y = m.y > 0.f ? g.y : 0.f;
        g.z = m.z > 0.f ? g.z : 0.f; g.w = m.w > 0.f ? g.w : 0.f;
        return g;
    }
};

__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(const BNArgs a) {
    __shared__ double red[4];
    const int s = blockIdx.x, c = blockIdx.y, z = blockIdx.z;
    const float mean = a.save_mean[z * a.C + c], invstd = a.save_invstd[z * a.C + c];
    const ReluMask rm(a, z, c, mean, invstd);
    const float* xz = a.x + z * a.x_cs;
    float* drz = a.dres ? a.dres + z * a.dres_cs : nullptr;
    double sg = 0.0, dot = 0.0;
    for_slice(a, z, c, s, [&](int64_t o, int nv) {
        if (nv == 4) {
            const float4 xv = ld4(xz + o);
            const float4 g = rm.apply4(upstream4(a, z, o), xv, o);
            if (drz) st4(drz + o, g);
            sg += ((double)g.x + (double)g.y) + ((double)g.z + (double)g.w);
            dot += ((double)((xv.x - mean) * g.x) + (double)((xv.y - mean) * g.y)) +
                   ((double)((xv.z - mean) * g.z) + (double)((xv.w - mean) * g.w));
        } else {
            const float xv = xz[o];
            const float g = rm.keep(xv, o) ? upstream1(a, z, o) : 0.f;
            if (drz) drz[o] = g;
            sg += (double)g;
            dot += (double)((xv - mean) * g);
        }
    });
    sg = block_sum_256(sg, red);
    dot = block_sum_256(dot, red);
    if (threadIdx.x == 0) {
        double* p = a.part + ((((int64_t)z * a.C + c) * a.S) + s) * 2;
        p[0] = sg;
        p[1] = dot;
    }
}

__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(const BNArgs a) {
    const int s = blockIdx.x, c = blockIdx.y, z = blockIdx.z;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int64_t n = (int64_t)cnt * a.HW;
    double sg, dot;
    merge(a, z, c, sg, dot);
    const float mean = a.save_mean[z * a.C + c], invstd = a.save_invstd[z * a.C + c];
    if (s == 0 && threadIdx.x == 0) {
        if (a.dgamma) a.dgamma[z * a.g_cs + c] = (float)(dot * (double)invstd);
        if (a.dbeta) a.dbeta[z * a.g_cs + c] = (float)sg;
    }
    if (!a.dx) return;
    const ReluMask rm(a, z, c, mean, invstd);
    const float w = a.gamma[z * a.p_cs + c];
    const float k = n > 0 ? (float)(dot * (double)invstd * (double)invstd / (double)n) : 0.f;
    const float gm = n > 0 ? (float)(sg / (double)n) : 0.f;
    const float* xz = a.x + z * a.x_cs;
    float* dxz = a.dx + z * a.dx_cs;
    auto apply4 = [&](float4 g, float4 xv) {
        float4 r;
        r.x = (((g.x - gm) - (xv.x - mean) * k) * invstd) * w;
        r.y = (((g.y - gm) - (xv.y - mean) * k) * invstd) * w;
        r.z = (((g.z - gm) - (xv.z - mean) * k) * invstd) * w;
        r.w = (((g.w - gm) - (xv.w - mean) * k) * invstd) * w;
        return r;
    };
    if (a.vec) {
        // float4 path, two element quads per thread per iteration with every load issued
        // before the first store (dx may alias nothing the loop reads, but the compiler
        // cannot know: one quad per iteration left one HBM round trip per quad)
        const int e0 = s * a.chunk, e1 = min((int)n, e0 + a.chunk);
        const int64_t istride = (int64_t)a.C * a.HW, coff = (int64_t)c * a.HW;
        for (int e = e0 + threadIdx.x * 4; e < e1; e += 2 * 256 * 4) {
            const bool two = e + 256 * 4 < e1;
            uint32_t img, p;
            a.fd_hw.divmod(e, img, p);
            const int64_t oa = img * istride + coff + p;
            int64_t ob = oa;
            if (two) {
                a.fd_hw.divmod(e + 256 * 4, img, p);
                ob = img * istride + coff + p;
            }
            const float4 xa = ld4(xz + oa), xb = ld4(xz + ob);
            const float4 ua = upstream4(a, z, oa), ub = upstream4(a, z, ob);
            const float4 ra = apply4(rm.apply4(ua, xa, oa), xa);
            const float4 rb = apply4(rm.apply4(ub, xb, ob), xb);
            st4(dxz + oa, ra);
            if (two) st4(dxz + ob, rb);
        }
        return;
    }
    for_slice(a, z, c, s, [&](int64_t o, int nv) {
        if (nv == 4) {
            const float4 xv = ld4(xz + o);
            const float4 g = rm.apply4(upstream4(a, z, o), xv, o);
            st4(dxz + o, apply4(g, xv));
        } else {
            const float xv = xz[o];
            const float g = rm.keep(xv, o) ? upstream1(a, z, o) : 0.f;
            dxz[o] = (((g - gm) - (xv - mean) * k) * invstd) * w;
        }
    });
}

// ---------------------------------------------------------------------------
// r06: a split conv's reduction + the BatchNorm call after it as one launch (splitbn.h).
// One 1024-thread workgroup per (channel, client): its four 256-thread groups take the
// channel's 256-element tiles in turn — the slab summed in split order, the tile's statistics
// pair formed as splitk_epilogue_kernel forms it (wave sums, then (w0 + w1) + (w2 + w3)) — and
// wave 0 merges the tiles as merge() does.  Everything stored is bit-identical to the
// epilogue launch + bn_finalize / maxpool2_bnfin / bn_bwd_apply pair it replaces.
constexpr int kSbnTpt = 8;  // tiles per 256-thread group in flight per pass
// Every global load of these kernels is unconditional (indices clamped into the tensor, the
// value discarded by a select): a load under a branch is joined by a phi whose wait drains
// the memory pipe — one dependent round trip per load (r06 first version: 4-8 per pass).

struct SbnFwd {
    SplitBnRec r;
    BNArgs a;  // the finalize's parameters (gamma, beta, running / saved statistics, C, HW)
    float* scale;
    float* shift;
    int64_t s_cs;
    int ntile;
    FastDiv fd_sp;
    // 2x2 max-pool (+ dropout) of relu(y * scale + shift): maxpool2_bnfin_kernel's outputs
    int pool;
    float* y;
    int64_t y_cs;
    uint8_t* idx;
    int64_t i_cs;
    uint8_t* mask;
    int64_t m_cs;
    int H, W, drop_mode;
    FastDiv fd_ohw, fd_ow;
    float keep_prob, dscale;
    uint64_t seed_salt;
    const uint64_t* seed_dev;
};

struct SbnBwd {
    SplitBnRec r;
    BNArgs a;  // the apply's parameters (x, gamma, beta, saved statistics, dx, dgamma, dbeta)
    int ntile;
    FastDiv fd_sp, fd_pw;  // the DGRAD's plane (sp) and, pooled, its width
};

// Tile statistics without cross-lane trees per tile (r06 second version: 8 tiles x 2
// xor-butterflies of ds_bpermute per thread dominated the 16x16 launches).  The epilogue's
// tile pair is (w0 + w1) + (w2 + w3) over the tile's four 64-element chunks, each wN the
// xor-butterfly wave_sum — whose value is the fixed tree x[i] += x[i + h], h = 32, 16, ..., 1.
// The per-element values sit in LDS (v0; v1 or v0^2 for the second moment) and all 1024
// threads build every chunk's tree level by level in T: the same sums in the same order.
using SbnTree = double[2][kSbnMaxTiles * 4][16];

template <bool SQ>
__device__ __forceinline__ void sbn_tree(const float* v0, const float* v1, int nch, SbnTree& T) {
    const int tid = threadIdx.x;
    for (int it = tid; it < 2 * nch * 16; it += 1024) {  // levels h = 32 and 16 from LDS
        const int st = it >= nch * 16, rem = it - st * nch * 16, ch = rem >> 4, i = rem & 15;
        const int b = ch * 64 + i;
        double x0, x1, x2, x3;
        if (st == 0 || SQ) {
            x0 = v0[b]; x1 = v0[b + 32]; x2 = v0[b + 16]; x3 = v0[b + 48];
            if (st) { x0 = x0 * x0; x1 = x1 * x1; x2 = x2 * x2; x3 = x3 * x3; }
        } else {
            x0 = v1[b]; x1 = v1[b + 32]; x2 = v1[b + 16]; x3 = v1[b + 48];
        }
        T[st][ch][i] = (x0 + x1) + (x2 + x3);
    }
#pragma unroll
    for (int h = 8; h >= 1; h >>= 1) {
        __syncthreads();
        for (int it = tid; it < 2 * nch * h; it += 1024) {
            const int st = it >= nch * h, rem = it - st * nch * h, ch = rem / h, i = rem - ch * h;
            T[st][ch][i] = T[st][ch][i] + T[st][ch][i + h];
        }
    }
    __syncthreads();
}

// the tiles' statistics pairs -> (sum0, sum1) in wave 0 (merge()'s order)
__device__ __forceinline__ void sbn_merge(const SbnTree& T, int ntile, double& s0, double& s1) {
    s0 = 0.0;
    s1 = 0.0;
    for (int i = threadIdx.x & 63; i < ntile; i += 64) {
        s0 += (T[0][4 * i][0] + T[0][4 * i + 1][0]) + (T[0][4 * i + 2][0] + T[0][4 * i + 3][0]);
        s1 += (T[1][4 * i][0] + T[1][4 * i + 1][0]) + (T[1][4 * i + 2][0] + T[1][4 * i + 3][0]);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
}

// this thread's kSbnTpt slab values per split (clamped loads; splits <= 4)
__device__ __forceinline__ void sbn_load_slab(const SplitBnRec& r, const float* pz, int64_t ss,
                                              int t0, int grp, int lt, float (&v)[kSbnTpt][4]) {
    const int nlast = (int)r.Nfull - 1, jl = r.splits - 1;
#pragma unroll
    for (int k = 0; k < kSbnTpt; ++k) {
        const int nc = min((t0 + 4 * k + grp) * 256 + lt, nlast);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = pz[min(j, jl) * ss + nc];
    }
}

// splitk_epilogue_kernel's sum: 0 + p0 + p1 + ... in split order
__device__ __forceinline__ float sbn_sum(const float (&v)[4], int splits) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (j < splits) s += v[j];
    return s;
}

__global__ void __launch_bounds__(1024) split_bnfin_kernel(const SbnFwd f) {
    __shared__ float ybuf[kSbnMaxElems];  // y, zero past the client's images
    __shared__ SbnTree T;
    __shared__ float s_aff[2];
    const SplitBnRec& r = f.r;
    const BNArgs& a = f.a;
    const int c = blockIdx.x, z = blockIdx.y;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int nvalid = cnt * r.sp;
    const int tid = threadIdx.x, grp = tid >> 8, lt = tid & 255, lane = tid & 63;
    const float* pz = r.part + ((int64_t)z * r.splits * r.M + c) * r.Nfull;
    const int64_t ss = (int64_t)r.M * r.Nfull;
    const float bv = r.bias ? r.bias[z * r.b_cs + c] : 0.f;
    float* oz = r.out + z * r.out_cs;
    for (int t0 = 0; t0 < f.ntile; t0 += 4 * kSbnTpt) {
        float v[kSbnTpt][4];
        sbn_load_slab(r, pz, ss, t0, grp, lt, v);
#pragma unroll
        for (int k = 0; k < kSbnTpt; ++k) {
            const int t = t0 + 4 * k + grp;
            if (t >= f.ntile) break;  // uniform over the 256-thread group
            const int n = t * 256 + lt;
            const bool ok = n < nvalid;
            float s = sbn_sum(v[k], r.splits);
            if (r.bias) s = s + bv;
            if (ok) {
                uint32_t img, pix;
                f.fd_sp.divmod((uint32_t)n, img, pix);
                oz[((int64_t)img * r.M + c) * r.sp + pix] = s;
            }
            ybuf[n] = ok ? s : 0.f;
        }
    }
    __syncthreads();
    sbn_tree<true>(ybuf, nullptr, 4 * f.ntile, T);
    if (tid < 64) {  // bn_finalize_kernel's operations
        double sum, sq;
        sbn_merge(T, f.ntile, sum, sq);
        if (lane == 0) {
            const int64_t n = (int64_t)cnt * a.HW;
            const double mean = n > 0 ? sum / (double)n : 0.0;
            double var = n > 0 ? sq / (double)n - mean * mean : 0.0;
            if (var < 0.0) var = 0.0;
            const double invstd = n > 0 ? 1.0 / sqrt(var + (double)a.eps) : 0.0;
            const float meanf = (float)mean, invstdf = (float)invstd;
            a.save_mean[z * a.C + c] = meanf;
            a.save_invstd[z * a.C + c] = invstdf;
            if (a.rmean && n > 0) {
                const double unb = n > 1 ? var * (double)n / (double)(n - 1) : var;
                float* rm = a.rmean + z * a.r_cs + c;
                float* rv = a.rvar + z * a.r_cs + c;
                *rm = (float)((double)a.momentum * mean + (1.0 - (double)a.momentum) * (double)*rm);
                *rv = (float)((double)a.momentum * unb + (1.0 - (double)a.momentum) * (double)*rv);
            }
            const float alpha = invstdf * a.gamma[z * a.p_cs + c];
            const float bconst = a.beta[z * a.p_cs + c] - meanf * alpha;
            f.scale[z * f.s_cs + c] = alpha;
            f.shift[z * f.s_cs + c] = bconst;
            s_aff[0] = alpha;
            s_aff[1] = bconst;
        }
    }
    if (!f.pool) return;  // launch-uniform
    __syncthreads();
    // maxpool2_bnfin_kernel's pool of relu(y * alpha + beta') from the tile values in LDS
    const float s = s_aff[0], t = s_aff[1];
    const int ohw = (f.H / 2) * (f.W / 2);
    const uint64_t seed = f.seed_salt + (f.seed_dev ? *f.seed_dev : 0ull);
    const uint64_t prow = f.drop_mode == 1 ? philox_row(f.seed_dev, z) : 0ull;
    for (int q = tid; q < cnt * ohw; q += 1024) {
        uint32_t img, rr, oh, ow;
        f.fd_ohw.divmod((uint32_t)q, img, rr);
        f.fd_ow.divmod(rr, oh, ow);
        const int64_t e = ((int64_t)img * a.C + c) * ohw + rr;
        const float* pp = ybuf + img * a.HW + (2 * oh) * f.W + 2 * ow;
        const float v0 = fmaxf(pp[0] * s + t, 0.f), v1 = fmaxf(pp[1] * s + t, 0.f);
        const float v2 = fmaxf(pp[f.W] * s + t, 0.f), v3 = fmaxf(pp[f.W + 1] * s + t, 0.f);
        float m = v0;
        int am = 0;
        if (v1 > m) { m = v1; am = 1; }
        if (v2 > m) { m = v2; am = 2; }
        if (v3 > m) { m = v3; am = 3; }
        f.idx[z * f.i_cs + e] = (uint8_t)am;
        if (f.drop_mode) {
            uint8_t keep;
            if (f.drop_mode == 1) {
                const uint4 rn = Philox::gen(seed, prow, (uint64_t)e);
                keep = u01(rn.x) <= f.keep_prob ? 1 : 0;
                f.mask[z * f.m_cs + e] = keep;
            } else {
                keep = f.mask[z * f.m_cs + e];
            }
            m = keep ? m * f.dscale : 0.f;
        }
        f.y[z * f.y_cs + e] = m;
    }
}

// Q: float4 quads per thread of the apply pass (cnt * HW <= Q * 4096), prefetched before the
// statistics merge so their loads overlap it
template <int Q, bool POOLED>
__global__ void __launch_bounds__(1024) split_bnbwd_kernel(const SbnBwd b) {
    __shared__ float gs[kSbnMaxElems];  // the masked gradient g (zero past the images)
    __shared__ float ps[kSbnMaxElems];  // (x - mean) * g
    __shared__ float gbuf[POOLED ? kSbnMaxElems : 1];    // pooled: the routed value gu
    __shared__ uint8_t cbuf[POOLED ? kSbnMaxElems : 1];  // pooled: window argmax
    __shared__ SbnTree T;
    __shared__ double s_st[2];
    const SplitBnRec& r = b.r;
    const BNArgs& a = b.a;
    const int c = blockIdx.x, z = blockIdx.y;
    const int cnt = a.counts ? a.counts[z] : a.batch;
    const int nvalid = cnt * r.sp;
    const int tid = threadIdx.x, grp = tid >> 8, lt = tid & 255, lane = tid & 63;
    constexpr bool pooled = POOLED;
    const float* pz = r.part + ((int64_t)z * r.splits * r.M + c) * r.Nfull;
    const int64_t ss = (int64_t)r.M * r.Nfull;
    const float esc = r.bn_scale[z * r.bns_cs + c], esh = r.bn_shift[z * r.bns_cs + c];
    const float emean = r.bn_mean[z * r.M + c];
    const float* bx = r.bnx + z * r.bnx_cs;
    // pooled: the keep-mask if any, else the argmax bytes again (a valid read, ignored)
    const uint8_t* pk = !POOLED ? nullptr : r.pmask ? r.pmask + z * r.pm_cs : r.pidx + z * r.pi_cs;
    const bool km = r.pmask != nullptr;
    const int nlast = (int)r.Nfull - 1;
    for (int t0 = 0; t0 < b.ntile; t0 += 4 * kSbnTpt) {
        float v[kSbnTpt][4], xv[kSbnTpt];
        int code[kSbnTpt];
        bool keep[kSbnTpt];
        sbn_load_slab(r, pz, ss, t0, grp, lt, v);
#pragma unroll
        for (int k = 0; k < kSbnTpt; ++k) {
            const int nc = min((t0 + 4 * k + grp) * 256 + lt, nlast);
            uint32_t img, pix;
            b.fd_sp.divmod((uint32_t)nc, img, pix);
            const int64_t e = ((int64_t)img * r.M + c) * r.sp + pix;
            if constexpr (POOLED) {
                code[k] = r.pidx[z * r.pi_cs + e];
                keep[k] = (pk[e] != 0) | !km;
                xv[k] = 0.f;
            } else {
                code[k] = 0;
                keep[k] = true;
                xv[k] = bx[e];
            }
        }
        if constexpr (POOLED) {  // the BN input at each window's argmax (splitk_epilogue_kernel's read)
#pragma unroll
            for (int k = 0; k < kSbnTpt; ++k) {
                const int nc = min((t0 + 4 * k + grp) * 256 + lt, nlast);
                uint32_t img, pix, py, px;
                b.fd_sp.divmod((uint32_t)nc, img, pix);
                b.fd_pw.divmod(pix, py, px);
                xv[k] = bx[((int64_t)img * r.M + c) * 4 * r.sp +
                           (2 * py + (code[k] >> 1)) * (2 * r.pw) + 2 * px + (code[k] & 1)];
            }
        }
#pragma unroll
        for (int k = 0; k < kSbnTpt; ++k) {
            const int t = t0 + 4 * k + grp;
            if (t >= b.ntile) break;  // uniform over the 256-thread group
            const int n = t * 256 + lt;
            const bool ok = n < nvalid;
            const float s = sbn_sum(v[k], r.splits);
            float gu = s;
            if (pooled && r.pmask) gu = keep[k] ? s * r.pscale : 0.f;
            const float g = (xv[k] * esc + esh > 0.f) ? gu : 0.f;
            const float d1f = (xv[k] - emean) * g;
            gs[n] = ok ? g : 0.f;
            ps[n] = ok ? d1f : 0.f;
            if constexpr (POOLED) {
                gbuf[n] = gu;
                cbuf[n] = (uint8_t)code[k];
            }
        }
    }
    // the apply pass's x, in flight across the merge
    const int ntot = cnt * a.HW;
    const float* xz = a.x + z * a.x_cs;
    const int64_t istride = (int64_t)a.C * a.HW, coff = (int64_t)c * a.HW;
    float4 xq[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        const int e = max(min(tid * 4 + i * 4096, ntot - 4), 0);
        uint32_t img, p;
        a.fd_hw.divmod((uint32_t)e, img, p);
        xq[i] = ld4(xz + img * istride + coff + p);
    }
    __syncthreads();
    sbn_tree<false>(gs, ps, 4 * b.ntile, T);
    if (tid < 64) {
        double sg, dot;
        sbn_merge(T, b.ntile, sg, dot);
        if (lane == 0) {
            s_st[0] = sg;
            s_st[1] = dot;
        }
    }
    __syncthreads();
    // bn_bwd_apply_kernel's operations over the channel's full-resolution elements
    const double sg = s_st[0], dot = s_st[1];
    const int64_t n = (int64_t)cnt * a.HW;
    const float mean = a.save_mean[z * a.C + c], invstd = a.save_invstd[z * a.C + c];
    if (tid == 0) {
        if (a.dgamma) a.dgamma[z * a.g_cs + c] = (float)(dot * (double)invstd);
        if (a.dbeta) a.dbeta[z * a.g_cs + c] = (float)sg;
    }
    if (!a.dx) return;
    const float w = a.gamma[z * a.p_cs + c];
    const float k = n > 0 ? (float)(dot * (double)invstd * (double)invstd / (double)n) : 0.f;
    const float gm = n > 0 ? (float)(sg / (double)n) : 0.f;
    float alpha = 0.f, bconst = 0.f;  // ReluMask mode 2 (pooled: recomputed from x)
    if (pooled) {
        alpha = invstd * a.gamma[z * a.p_cs + c];
        bconst = a.beta[z * a.p_cs + c] - mean * alpha;
    }
    float* dxz = a.dx + z * a.dx_cs;
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        const int e = tid * 4 + i * 4096;
        if (e >= ntot) break;
        uint32_t img, p;
        a.fd_hw.divmod((uint32_t)e, img, p);
        const int64_t o = img * istride + coff + p;
        const float4 xv = xq[i];
        float4 g;
        if (pooled) {
            uint32_t y, x;
            a.fd_w.divmod(p, y, x);
            const int pe = img * r.sp + (y >> 1) * r.pw + (x >> 1);
            const int c0 = cbuf[pe], c1 = cbuf[pe + 1];
            const float g0 = gbuf[pe], g1 = gbuf[pe + 1];
            const int rr = (y & 1) << 1;
            g = make_float4(c0 == rr ? g0 : 0.f, c0 == (rr | 1) ? g0 : 0.f, c1 == rr ? g1 : 0.f,
                            c1 == (rr | 1) ? g1 : 0.f);
            float4 m;
            m.x = xv.x * alpha + bconst; m.y = xv.y * alpha + bconst;
            m.z = xv.z * alpha + bconst; m.w = xv.w * alpha + bconst;
            g.x = m.x > 0.f ? g.x : 0.f; g.y = m.y > 0.f ? g.y : 0.f;
            g.z = m.z > 0.f ? g.z : 0.f; g.w = m.w > 0.f ? g.w : 0.f;
        } else {
            g = make_float4(gs[e], gs[e + 1], gs[e + 2], gs[e + 3]);
        }
        float4 rv;
        rv.x = (((g.x - gm) - (xv.x - mean) * k) * invstd) * w;
        rv.y = (((g.y - gm) - (xv.y - mean) * k) * invstd) * w;
        rv.z = (((g.z - gm) - (xv.z - mean) * k) * invstd) * w;
        rv.w = (((g.w - gm) - (xv.w - mean) * k) * invstd) * w;
        st4(dxz + o, rv);
    }
}

// the apply pass's quads per thread: 2 (<= 8192 elements per client-channel) or 8 (<= 32768)
static int sbn_bwd_launch(SbnBwd& b, int C, int nclients, int batch, int HW, hipStream_t st) {
    b.fd_sp = FastDiv((uint32_t)b.r.sp);
    b.fd_pw = FastDiv((uint32_t)std::max(b.r.pw, 1));
    const bool pooled = b.r.pidx != nullptr;
    if ((int64_t)batch * HW <= 2 * 4096) {
        if (pooled)
            FH_LAUNCH((split_bnbwd_kernel<2, true>), dim3((unsigned)C, nclients), dim3(1024), 0, st, b);
        else
            FH_LAUNCH((split_bnbwd_kernel<2, false>), dim3((unsigned)C, nclients), dim3(1024), 0, st, b);
    } else {
        FH_REQUIRE(pooled && (int64_t)batch * HW <= 8 * 4096, "split bn backward: %d x %d", batch, HW);
        FH_LAUNCH((split_bnbwd_kernel<8, true>), dim3((unsigned)C, nclients), dim3(1024), 0, st, b);
    }
    return FH_OK;
}

// fused launches issued (fh_conv_bn_defer_status)
thread_local int64_t g_sbn_taken = 0;

// a pending split record nobody here consumes: launch its epilogue first
static int sbn_settle() { return sbn_rec().pending ? sbn_materialize() : FH_OK; }

int64_t sbn_taken() { return g_sbn_taken; }

static void bn_geometry(int nclients, int batch, int C, int HW, int& S, int& chunk) {
    const int64_t nmax = (int64_t)batch * HW;
    int64_t want = ceil_div(2048, (int64_t)C * std::max(nclients, 1));
    const int64_t maxs = std::max<int64_t>(1, nmax / 2048);  // >= 2048 elements per slice
    if (want > maxs) want = maxs;
    if (want < 1) want = 1;
    chunk = (int)(ceil_div(ceil_div(nmax, want), 4) * 4);
    S = (int)ceil_div(nmax, chunk);
}

static BNArgs bn_args(int nclients, int batch, int C, int HW, const int32_t* counts) {
    BNArgs a{};
    a.counts = counts;
    a.batch = batch;
    a.C = C;
    a.HW = HW;
    bn_geometry(nclients, batch, C, HW, a.S, a.chunk);
    a.SP = a.S;
    a.fd_hw = FastDiv(HW);
    a.vec = (HW & 3) == 0;
    return a;
}

}  // namespace fh

using namespace fh;

extern "C" size_t fh_bn_workspace(int32_t nclients, int32_t batch, int32_t C, int32_t HW) {
    if (nclients <= 0 || batch <= 0 || C <= 0 || HW <= 0) return 0;
    int S, chunk;
    bn_geometry(nclients, batch, C, HW, S, chunk);
    return (size_t)nclients * C * S * 2 * sizeof(double);
}

extern "C" int fh_bn_fwd_train(const float* x, int64_t x_cs, float* y, int64_t y_cs,
                               const float* res, int64_t res_cs, const float* gamma,
                               const float* beta, int64_t p_cs, float* running_mean,
                               float* running_var, int64_t r_cs, float* save_mean,
                               float* save_invstd, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t C, int32_t HW, float eps, float momentum,
                               int32_t relu, void* workspace, size_t ws_bytes, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_fwd_train: bad shape");
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(x && y && gamma && beta && save_mean && save_invstd, "bn_fwd_train: null pointer");
    FH_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "bn_fwd_train: running stats");
    const size_t need = fh_bn_workspace(nclients, batch, C, HW);
    FH_REQUIRE(workspace && ws_bytes >= need, "bn_fwd_train: workspace %zu < %zu", ws_bytes, need);
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.x = x; a.y = y; a.res = res; a.gamma = gamma; a.beta = beta;
    a.rmean = running_mean; a.rvar = running_var; a.save_mean = save_mean;
    a.save_invstd = save_invstd; a.part = (double*)workspace;
    a.x_cs = x_cs; a.y_cs = y_cs; a.res_cs = res_cs; a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.momentum = momentum; a.relu = relu;
    hipStream_t st = as_stream(stream);
    dim3 grid(a.S, C, nclients);
    FH_LAUNCH(bn_stats_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_fwd_train stats");
    FH_LAUNCH(bn_apply_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_fwd_train apply");
    return FH_OK;
}

extern "C" int fh_bn_fwd_stats(const float* x, int64_t x_cs, const float* gamma,
                               const float* beta, int64_t p_cs, float* running_mean,
                               float* running_var, int64_t r_cs, float* save_mean,
                               float* save_invstd, float* scale_out, float* shift_out,
                               int64_t s_cs, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t C, int32_t HW, float eps, float momentum,
                               void* workspace, size_t ws_bytes, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_fwd_stats: bad shape");
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(x && gamma && beta && save_mean && save_invstd && scale_out && shift_out,
               "bn_fwd_stats: null pointer");
    FH_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "bn_fwd_stats: running stats");
    const size_t need = fh_bn_workspace(nclients, batch, C, HW);
    FH_REQUIRE(workspace && ws_bytes >= need, "bn_fwd_stats: workspace %zu < %zu", ws_bytes, need);
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.x = x; a.gamma = gamma; a.beta = beta;
    a.rmean = running_mean; a.rvar = running_var; a.save_mean = save_mean;
    a.save_invstd = save_invstd; a.part = (double*)workspace;
    a.x_cs = x_cs; a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.momentum = momentum;
    hipStream_t st = as_stream(stream);
    FH_LAUNCH(bn_stats_kernel, dim3(a.S, C, nclients), dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_fwd_stats stats");
    FH_LAUNCH(bn_finalize_kernel, dim3((unsigned)ceil_div(C, 4), nclients), dim3(256), 0,
                       st, a, scale_out, shift_out, s_cs);
    FH_LAUNCH_CHECK("bn_fwd_stats finalize");
    return FH_OK;
}

// Train-mode statistics from partials a convolution epilogue already wrote
// (fh_conv2d_fwd_bnstats: one fp64 (sum, sum of squares) pair per (client, channel,
// 256-pixel tile), zeros past a client's count): bn_finalize_kernel merges the tiles in
// order -> save_mean / save_invstd, running statistics, and the consumer's affine.
extern "C" int fh_bn_finalize_tiles(const double* part, const float* gamma, const float* beta,
                                    int64_t p_cs, float* running_mean, float* running_var,
                                    int64_t r_cs, float* save_mean, float* save_invstd,
                                    float* scale_out, float* shift_out, int64_t s_cs,
                                    const int32_t* counts, int32_t nclients, int32_t batch,
                                    int32_t C, int32_t HW, float eps, float momentum,
                                    void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_finalize_tiles: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(part && gamma && beta && save_mean && save_invstd && scale_out && shift_out,
               "bn_finalize_tiles: null pointer");
    FH_REQUIRE((running_mean == nullptr) == (running_var == nullptr),
               "bn_finalize_tiles: running stats");
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.S = a.SP = (int)ceil_div((int64_t)batch * HW, 256);
    a.part = (double*)part;
    a.gamma = gamma; a.beta = beta;
    a.rmean = running_mean; a.rvar = running_var; a.save_mean = save_mean;
    a.save_invstd = save_invstd;
    a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.momentum = momentum;
    SplitBnRec& r = sbn_rec();
    if (r.pending) {
        if (r.op == 0 && r.bn_part == part && r.st == as_stream(stream) && r.M == C &&
            r.sp == HW && r.nclients == nclients && r.batch == batch && r.counts == counts) {
            // the split conv's reduction and this finalize: one launch (splitbn.h)
            SbnFwd f{};
            f.r = r;
            f.a = a;
            f.scale = scale_out; f.shift = shift_out; f.s_cs = s_cs;
            f.ntile = a.SP;
            f.fd_sp = FastDiv((uint32_t)HW);
            r.pending = false;
            FH_LAUNCH(split_bnfin_kernel, dim3((unsigned)C, nclients), dim3(1024), 0,
                      as_stream(stream), f);
            FH_LAUNCH_CHECK("bn_finalize_tiles (split conv reduction)");
            ++g_sbn_taken;
            return FH_OK;
        }
        if (const int rc = sbn_materialize()) return rc;
    }
    FH_LAUNCH(bn_finalize_kernel, dim3((unsigned)ceil_div(C, 4), nclients), dim3(256), 0,
              as_stream(stream), a, scale_out, shift_out, s_cs);
    FH_LAUNCH_CHECK("bn_finalize_tiles");
    return FH_OK;
}

// fh_bn_fwd_train's apply pass from the per-tile statistics a convolution epilogue wrote
// (FederatedResNet's stem bn1 and block bn2, whose output is materialised because the next
// block reads it twice, conv and residual): bn_apply_kernel merges the conv tiles instead of
// bn_stats_kernel's slices -> y = [relu](x*alpha + beta' [+ res]), save_mean / save_invstd
// and the running statistics.  y is never re-read for its statistics.
extern "C" int fh_bn_apply_tiles(const double* part, const float* x, int64_t x_cs, float* y,
                                 int64_t y_cs, const float* res, int64_t res_cs,
                                 const float* gamma, const float* beta, int64_t p_cs,
                                 float* running_mean, float* running_var, int64_t r_cs,
                                 float* save_mean, float* save_invstd, const int32_t* counts,
                                 int32_t nclients, int32_t batch, int32_t C, int32_t HW,
                                 float eps, float momentum, int32_t relu, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_apply_tiles: bad shape");
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(part && x && y && gamma && beta && save_mean && save_invstd,
               "bn_apply_tiles: null pointer");
    FH_REQUIRE((running_mean == nullptr) == (running_var == nullptr),
               "bn_apply_tiles: running stats");
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.SP = (int)ceil_div((int64_t)batch * HW, 256);  // the conv epilogue's tiles
    a.part = (double*)part;
    a.x = x; a.y = y; a.res = res; a.gamma = gamma; a.beta = beta;
    a.rmean = running_mean; a.rvar = running_var; a.save_mean = save_mean;
    a.save_invstd = save_invstd;
    a.x_cs = x_cs; a.y_cs = y_cs; a.res_cs = res_cs; a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.momentum = momentum; a.relu = relu;
    FH_LAUNCH(bn_apply_kernel, dim3(a.S, C, nclients), dim3(256), 0, as_stream(stream), a);
    FH_LAUNCH_CHECK("bn_apply_tiles");
    return FH_OK;
}

// fh_bn_finalize_tiles + fh_maxpool2_fwd_bnrelu in one launch (maxpool2_bnfin_kernel).
extern "C" int fh_maxpool2_fwd_bnfinalize(
        const double* part, const float* gamma, const float* beta, int64_t p_cs,
        float* running_mean, float* running_var, int64_t r_cs, float* save_mean,
        float* save_invstd, float* scale_out, float* shift_out, int64_t s_cs, const float* x,
        int64_t x_cs, float* y, int64_t y_cs, uint8_t* idx, int64_t i_cs, uint8_t* mask,
        int64_t m_cs, const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
        int32_t H, int32_t W, float eps, float momentum, int32_t drop_mode, float p_drop,
        uint64_t seed, const uint64_t* seed_dev, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && H >= 2 && W >= 2 && !(H & 1) && !(W & 1),
               "maxpool2_fwd_bnfinalize: bad shape");
    FH_REQUIRE(drop_mode >= 0 && drop_mode <= 2 && (drop_mode == 0 || mask),
               "maxpool2_fwd_bnfinalize: mask");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "maxpool2_fwd_bnfinalize: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(part && gamma && beta && save_mean && save_invstd && scale_out && shift_out && x &&
               y && idx, "maxpool2_fwd_bnfinalize: null pointer");
    FH_REQUIRE((running_mean == nullptr) == (running_var == nullptr),
               "maxpool2_fwd_bnfinalize: running stats");
    BNArgs a = bn_args(nclients, batch, C, H * W, counts);
    a.S = a.SP = (int)ceil_div((int64_t)batch * H * W, 256);
    a.part = (double*)part;
    a.gamma = gamma; a.beta = beta;
    a.rmean = running_mean; a.rvar = running_var; a.save_mean = save_mean;
    a.save_invstd = save_invstd;
    a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.momentum = momentum;
    const int64_t per_ch = (int64_t)batch * (H / 2) * (W / 2);
    const int bpc = (int)std::max<int64_t>(1, ceil_div(per_ch, 256 * kPoolEpt));
    const float keep = 1.0f - p_drop;
    SplitBnRec& r = sbn_rec();
    if (r.pending) {
        if (r.op == 0 && r.bn_part == part && r.st == as_stream(stream) && r.M == C &&
            r.sp == H * W && r.out == x && r.out_cs == x_cs && r.nclients == nclients &&
            r.batch == batch && r.counts == counts) {
            SbnFwd f{};
            f.r = r;
            f.a = a;
            f.scale = scale_out; f.shift = shift_out; f.s_cs = s_cs;
            f.ntile = a.SP;
            f.pool = 1;
            f.y = y; f.y_cs = y_cs; f.idx = idx; f.i_cs = i_cs; f.mask = mask; f.m_cs = m_cs;
            f.H = H; f.W = W; f.drop_mode = drop_mode; f.keep_prob = keep; f.dscale = 1.0f / keep;
            f.seed_salt = seed; f.seed_dev = seed_dev;
            f.fd_sp = FastDiv((uint32_t)(H * W));
            f.fd_ohw = FastDiv((uint32_t)((H / 2) * (W / 2)));
            f.fd_ow = FastDiv((uint32_t)(W / 2));
            r.pending = false;
            FH_LAUNCH(split_bnfin_kernel, dim3((unsigned)C, nclients), dim3(1024), 0,
                      as_stream(stream), f);
            FH_LAUNCH_CHECK("maxpool2_fwd_bnfinalize (split conv reduction)");
            ++g_sbn_taken;
            return FH_OK;
        }
        if (const int rc = sbn_materialize()) return rc;
    }
    FH_LAUNCH(maxpool2_bnfin_kernel, dim3((unsigned)(C * bpc), nclients), dim3(256), 0,
              as_stream(stream), a, scale_out, shift_out, s_cs, x, x_cs, y, y_cs, idx, i_cs,
              mask, m_cs, H, W, drop_mode, keep, 1.0f / keep, seed, seed_dev, bpc);
    FH_LAUNCH_CHECK("maxpool2_fwd_bnfinalize");
    return FH_OK;
}

extern "C" int fh_bn_fwd_eval(const float* x, int64_t x_cs, float* y, int64_t y_cs,
                              const float* res, int64_t res_cs, const float* gamma,
                              const float* beta, int64_t p_cs, const float* running_mean,
                              const float* running_var, int64_t r_cs, const int32_t* counts,
                              int32_t nclients, int32_t batch, int32_t C, int32_t HW, float eps,
                              int32_t relu, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_fwd_eval: bad shape");
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(x && y && gamma && beta && running_mean && running_var, "bn_fwd_eval: null pointer");
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.x = x; a.y = y; a.res = res; a.gamma = gamma; a.beta = beta;
    a.rmean = (float*)running_mean; a.rvar = (float*)running_var;
    a.x_cs = x_cs; a.y_cs = y_cs; a.res_cs = res_cs; a.p_cs = p_cs; a.r_cs = r_cs;
    a.eps = eps; a.relu = relu;
    FH_LAUNCH(bn_eval_kernel, dim3(a.S, C, nclients), dim3(256), 0, as_stream(stream), a);
    FH_LAUNCH_CHECK("bn_fwd_eval");
    return FH_OK;
}

extern "C" int fh_bn_bwd(const float* dy, int64_t dy_cs, const float* yout, int64_t yo_cs,
                         const float* x, int64_t x_cs, const float* gamma, const float* beta,
                         int64_t p_cs,
                         const float* save_mean, const float* save_invstd, float* dx,
                         int64_t dx_cs, float* dres, int64_t dres_cs, float* dgamma, float* dbeta,
                         int64_t g_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                         int32_t C, int32_t HW, int32_t relu, void* workspace, size_t ws_bytes,
                         void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_bwd: bad shape");
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(dy && x && gamma && save_mean && save_invstd, "bn_bwd: null pointer");
    FH_REQUIRE(!relu || yout || beta, "bn_bwd: relu needs the forward output or beta");
    const size_t need = fh_bn_workspace(nclients, batch, C, HW);
    FH_REQUIRE(workspace && ws_bytes >= need, "bn_bwd: workspace %zu < %zu", ws_bytes, need);
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.dy = dy; a.yout = yout; a.x = x; a.gamma = gamma; a.beta = beta;
    a.save_mean = (float*)save_mean;
    a.save_invstd = (float*)save_invstd; a.dx = dx; a.dres = dres; a.dgamma = dgamma;
    a.dbeta = dbeta; a.part = (double*)workspace;
    a.dy_cs = dy_cs; a.yo_cs = yo_cs; a.x_cs = x_cs; a.p_cs = p_cs; a.dx_cs = dx_cs;
    a.dres_cs = dres_cs; a.g_cs = g_cs; a.relu = relu;
    hipStream_t st = as_stream(stream);
    dim3 grid(a.S, C, nclients);
    FH_LAUNCH(bn_bwd_reduce_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_bwd reduce");
    FH_LAUNCH(bn_bwd_apply_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_bwd apply");
    return FH_OK;
}

// BN backward whose upstream gradient arrives through MaxPool2d(2,2) (+ the Dropout fused
// after it): the full-resolution gradient is routed on the fly from dpool / pidx / pmask
// (maxpool2_bwd semantics) instead of being written and re-read.
extern "C" int fh_bn_bwd_pool(const float* dpool, int64_t dp_cs, const uint8_t* pidx,
                              int64_t pi_cs, const uint8_t* pmask, int64_t pm_cs, float p_drop,
                              const float* yout, int64_t yo_cs, const float* x, int64_t x_cs,
                              const float* gamma, const float* beta, int64_t p_cs,
                              const float* save_mean,
                              const float* save_invstd, float* dx, int64_t dx_cs, float* dgamma,
                              float* dbeta, int64_t g_cs, const int32_t* counts,
                              int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                              int32_t relu, void* workspace, size_t ws_bytes, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && H >= 2 && W >= 2 && !(H & 1) && !(W & 1),
               "bn_bwd_pool: bad shape");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "bn_bwd_pool: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    if (const int rc = sbn_settle()) return rc;
    FH_REQUIRE(dpool && pidx && x && gamma && save_mean && save_invstd, "bn_bwd_pool: null pointer");
    FH_REQUIRE(!relu || yout || beta, "bn_bwd_pool: relu needs the forward output or beta");
    const int HW = H * W;
    const size_t need = fh_bn_workspace(nclients, batch, C, HW);
    FH_REQUIRE(workspace && ws_bytes >= need, "bn_bwd_pool: workspace %zu < %zu", ws_bytes, need);
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.dpool = dpool; a.pidx = pidx; a.pmask = pmask;
    a.dp_cs = dp_cs; a.pi_cs = pi_cs; a.pm_cs = pm_cs;
    a.pscale = 1.0f / (1.0f - p_drop);
    a.W = W;
    a.fd_w = FastDiv(W);
    a.vec = (HW & 3) == 0 && (W & 3) == 0;
    a.yout = yout; a.x = x; a.gamma = gamma; a.beta = beta; a.save_mean = (float*)save_mean;
    a.save_invstd = (float*)save_invstd; a.dx = dx; a.dgamma = dgamma; a.dbeta = dbeta;
    a.part = (double*)workspace;
    a.yo_cs = yo_cs; a.x_cs = x_cs; a.p_cs = p_cs; a.dx_cs = dx_cs; a.g_cs = g_cs; a.relu = relu;
    hipStream_t st = as_stream(stream);
    dim3 grid(a.S, C, nclients);
    FH_LAUNCH(bn_bwd_reduce_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_bwd_pool reduce");
    FH_LAUNCH(bn_bwd_apply_kernel, grid, dim3(256), 0, st, a);
    FH_LAUNCH_CHECK("bn_bwd_pool apply");
    return FH_OK;
}

// BN backward from statistics a convolution's DGRAD epilogue already took
// (fh_conv2d_dgrad_bnstats: g is the ReLU-masked gradient, bn_part holds one fp64
// (sum g, sum (x - mean) g) pair per (client, channel, 256-pixel tile)): the apply pass of
// fh_bn_bwd only — dgamma / dbeta and dx = ((g - mean g) - (x - mean) k) invstd w.
extern "C" int fh_bn_bwd_tiles(const double* part, const float* g, int64_t g_cs_, const float* x,
                               int64_t x_cs, const float* gamma, int64_t p_cs,
                               const float* save_mean, const float* save_invstd, float* dx,
                               int64_t dx_cs, float* dgamma, float* dbeta, int64_t dg_cs,
                               const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                               int32_t HW, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && HW > 0, "bn_bwd_tiles: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(part && g && x && gamma && save_mean && save_invstd, "bn_bwd_tiles: null pointer");
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.SP = (int)ceil_div((int64_t)batch * HW, 256);
    a.part = (double*)part;
    a.dy = g; a.x = x; a.gamma = gamma;
    a.save_mean = (float*)save_mean; a.save_invstd = (float*)save_invstd;
    a.dx = dx; a.dgamma = dgamma; a.dbeta = dbeta;
    a.dy_cs = g_cs_; a.x_cs = x_cs; a.p_cs = p_cs; a.dx_cs = dx_cs; a.g_cs = dg_cs;
    a.relu = 0;  // g is already masked
    SplitBnRec& r = sbn_rec();
    if (r.pending) {
        if (r.op == 1 && !r.pidx && r.bn_part == part && r.st == as_stream(stream) && r.M == C &&
            r.sp == HW && r.out == g && r.out_cs == g_cs_ && r.nclients == nclients &&
            r.batch == batch && r.counts == counts && a.vec) {
            // the split DGRAD's reduction + its BN-backward statistics and this apply: one
            // launch; g itself is never stored (only this apply read it)
            SbnBwd b{};
            b.r = r;
            b.a = a;
            b.ntile = a.SP;
            r.pending = false;
            if (const int rc = sbn_bwd_launch(b, C, nclients, batch, HW, as_stream(stream)))
                return rc;
            FH_LAUNCH_CHECK("bn_bwd_tiles (split conv reduction)");
            ++g_sbn_taken;
            return FH_OK;
        }
        if (const int rc = sbn_materialize()) return rc;
    }
    FH_LAUNCH(bn_bwd_apply_kernel, dim3(a.S, C, nclients), dim3(256), 0, as_stream(stream), a);
    FH_LAUNCH_CHECK("bn_bwd_tiles");
    return FH_OK;
}

// fh_bn_bwd_pool's apply pass from the partials fh_conv2d_dgrad_bnstats took with pidx (the
// statistics over the pooled grid's tiles, routed to the window argmax): dgamma / dbeta and
// dx, the gradient routed from dpool / pidx / pmask and the ReLU mask recomputed from x.
extern "C" int fh_bn_bwd_pool_tiles(const double* part, const float* dpool, int64_t dp_cs,
                                    const uint8_t* pidx, int64_t pi_cs, const uint8_t* pmask,
                                    int64_t pm_cs, float p_drop, const float* x, int64_t x_cs,
                                    const float* gamma, const float* beta, int64_t p_cs,
                                    const float* save_mean, const float* save_invstd, float* dx,
                                    int64_t dx_cs, float* dgamma, float* dbeta, int64_t g_cs,
                                    const int32_t* counts, int32_t nclients, int32_t batch,
                                    int32_t C, int32_t H, int32_t W, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && C > 0 && H >= 2 && W >= 2 && !(H & 1) && !(W & 1),
               "bn_bwd_pool_tiles: bad shape");
    FH_REQUIRE(p_drop >= 0.f && p_drop < 1.f, "bn_bwd_pool_tiles: p=%g", p_drop);
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(part && dpool && pidx && x && gamma && beta && save_mean && save_invstd,
               "bn_bwd_pool_tiles: null pointer");
    const int HW = H * W;
    BNArgs a = bn_args(nclients, batch, C, HW, counts);
    a.SP = (int)ceil_div((int64_t)batch * (HW / 4), 256);
    a.part = (double*)part;
    a.dpool = dpool; a.pidx = pidx; a.pmask = pmask;
    a.dp_cs = dp_cs; a.pi_cs = pi_cs; a.pm_cs = pm_cs;
    a.pscale = 1.0f / (1.0f - p_drop);
    a.W = W;
    a.fd_w = FastDiv(W);
    a.vec = (HW & 3) == 0 && (W & 3) == 0;
    a.x = x; a.gamma = gamma; a.beta = beta; a.save_mean = (float*)save_mean;
    a.save_invstd = (float*)save_invstd; a.dx = dx; a.dgamma = dgamma; a.dbeta = dbeta;
    a.x_cs = x_cs; a.p_cs = p_cs; a.dx_cs = dx_cs; a.g_cs = g_cs; a.relu = 1;
    SplitBnRec& r = sbn_rec();
    if (r.pending) {
        if (r.op == 1 && r.pidx == pidx && r.pmask == pmask && r.pi_cs == pi_cs &&
            r.pm_cs == pm_cs && r.pscale == a.pscale && r.bn_part == part &&
            r.st == as_stream(stream) && r.M == C && 4 * r.sp == HW && 2 * r.pw == W &&
            r.out == dpool && r.out_cs == dp_cs && r.nclients == nclients && r.batch == batch &&
            r.counts == counts && a.vec) {
            SbnBwd b{};
            b.r = r;
            b.a = a;
            b.ntile = a.SP;
            r.pending = false;
            if (const int rc = sbn_bwd_launch(b, C, nclients, batch, HW, as_stream(stream)))
                return rc;
            FH_LAUNCH_CHECK("bn_bwd_pool_tiles (split conv reduction)");
            ++g_sbn_taken;
            return FH_OK;
        }
        if (const int rc = sbn_materialize()) return rc;
    }
    FH_LAUNCH(bn_bwd_apply_kernel, dim3(a.S, C, nclients), dim3(256), 0, as_stream(stream), a);
    FH_LAUNCH_CHECK("bn_bwd_pool_tiles");
    return FH_OK;
}
