// optim.hip — optimizer steps over the packed [clients][P] parameter rows.
//
// Reference: LocalTrainer._create_optimizer (src/shared/training.py:244-255)
//   'sgd'   -> torch.optim.SGD(lr, momentum=0.9)
//   'adam'  -> torch.optim.Adam(lr)               (betas .9/.999, eps 1e-8)
//   'adamw' -> torch.optim.AdamW(lr)              (weight_decay 0.01)
// and the step is torch.optim's single-tensor CPU path.  The rounding
// sequence below follows ATen's CPU kernels for those tensor ops:
//   add(.., alpha)  -> fmadd(b, alpha, a)     lerp (w<.5) -> fmadd(w, e-s, s)
//   addcmul         -> a + (v*b)*c            addcdiv     -> a + v*(b/c)
// The optimizer is re-created every round (training.py:89), so callers pass
// first_step / step counts that restart at 1 each round.
#include "fh_common.h"

namespace fh {

__global__ void __launch_bounds__(256)
sgd_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ buf, int64_t n,
           float neg_lr, float mom, float wd, int first) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float pv = p[i];
        float gv = g[i];
        if (wd != 0.f) gv = fmaf(pv, wd, gv);
        float b;
        if (mom != 0.f) {
            b = first ? gv : (buf[i] * mom + gv);
            buf[i] = b;
        } else {
            b = gv;
        }
        p[i] = fmaf(b, neg_lr, pv);
    }
}

// The same update, four parameters per lane (16-B loads/stores; rows are 256-B aligned and
// padded to 64 floats, so packed slabs always qualify).  Per-element arithmetic is the
// scalar kernel's, so both give identical bits.
__device__ __forceinline__ float sgd_elem(float pv, float gv, float bv, float neg_lr, float mom,
                                          float wd, int first, float& b_out) {
    if (wd != 0.f) gv = fmaf(pv, wd, gv);
    float b = gv;
    if (mom != 0.f) b = first ? gv : (bv * mom + gv);
    b_out = b;
    return fmaf(b, neg_lr, pv);
}

__global__ void __launch_bounds__(256)
sgd4_kernel(float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ buf,
            int64_t n4, float neg_lr, float mom, float wd, int first) {
    const bool use_buf = mom != 0.f;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float4 pv = p[i];
        const float4 gv = g[i];
        const float4 bv = (use_buf && !first) ? buf[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 b, o;
        o.x = sgd_elem(pv.x, gv.x, bv.x, neg_lr, mom, wd, first, b.x);
        o.y = sgd_elem(pv.y, gv.y, bv.y, neg_lr, mom, wd, first, b.y);
        o.z = sgd_elem(pv.z, gv.z, bv.z, neg_lr, mom, wd, first, b.z);
        o.w = sgd_elem(pv.w, gv.w, bv.w, neg_lr, mom, wd, first, b.w);
        if (use_buf) buf[i] = b;
        p[i] = o;
    }
}

// One Adam/AdamW element in torch.optim's rounding order; shared by the scalar and the
// float4 kernel so the two give identical bits.
__device__ __forceinline__ float adam_elem(float pv, float gv, float& m, float& v, float wd,
                                          float decay_mul, int decoupled, float one_m_b1,
                                          float b2, float one_m_b2, float bc2_sqrt, float eps,
                                          float neg_step_size) {
    if (wd != 0.f) {
        if (decoupled) pv = pv * decay_mul;
        else gv = fmaf(pv, wd, gv);
    }
    const float mv = fmaf(one_m_b1, gv - m, m);
    const float vv = v * b2 + (one_m_b2 * gv) * gv;
    m = mv;
    v = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    return pv + neg_step_size * (mv / denom);
}

__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
            float* __restrict__ v, int64_t n, float wd, float decay_mul, int decoupled,
            float one_m_b1, float b2, float one_m_b2, float bc2_sqrt_h, float eps,
            float neg_step_size_h, const float* __restrict__ scal) {
    // per-step bias corrections: host scalars, or [bc2_sqrt, -step_size] in device memory
    // (lets one captured step graph serve every optimizer step)
    const float bc2_sqrt = scal ? scal[0] : bc2_sqrt_h;
    const float neg_step_size = scal ? scal[1] : neg_step_size_h;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        float mv = m[i], vv = v[i];
        p[i] = adam_elem(p[i], g[i], mv, vv, wd, decay_mul, decoupled, one_m_b1, b2, one_m_b2,
                         bc2_sqrt, eps, neg_step_size);
        m[i] = mv;
        v[i] = vv;
    }
}

__global__ void __launch_bounds__(256)
adam4_kernel(float4* __restrict__ p, const float4* __restrict__ g, float4* __restrict__ m,
             float4* __restrict__ v, int64_t n4, float wd, float decay_mul, int decoupled,
             float one_m_b1, float b2, float one_m_b2, float bc2_sqrt_h, float eps,
             float neg_step_size_h, const float* __restrict__ scal) {
    const float bc2_sqrt = scal ? scal[0] : bc2_sqrt_h;
    const float neg_step_size = scal ? scal[1] : neg_step_size_h;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * blockDim.x) {
        const float4 pv = p[i], gv = g[i];
        float4 mv = m[i], vv = v[i], o;
#define FH_ADAM_LANE(c) o.c = adam_elem(pv.c, gv.c, mv.c, vv.c, wd, decay_mul, decoupled, \
                                        one_m_b1, b2, one_m_b2, bc2_sqrt, eps, neg_step_size)
        FH_ADAM_LANE(x); FH_ADAM_LANE(y); FH_ADAM_LANE(z); FH_ADAM_LANE(w);
#undef FH_ADAM_LANE
        m[i] = mv;
        v[i] = vv;
        p[i] = o;
    }
}

// ---- optimizer steps that finish split WGRAD reductions (r03) --------------------------
// The row is cut into ranges: slab ranges (a convolution's weight or bias gradient still
// split over pixel ranges, fh_conv2d_wgrad_deferred) and the plain ranges between them.
// blockIdx.y = client, blockIdx.x walks the ranges' blocks (blk0 = a range's first block).
// A slab block is conv.hip splitk_sum_kernel<G> line for line — a thread owns one float4 of
// outputs and one of G contiguous split ranges, 8 loads in flight, the G range sums added in
// range order through LDS, G chosen from the split count as splitk_sum does — so g has the
// bits the separate reduction launch gave; g is stored and the update applied in place.
// A plain block reads g and updates 1024 float4s.  The separate reduction launch, its write
// of g and the optimizer's read of g disappear for every split layer.
struct SlabRange {
    int off4, len4;       // float4s within a row
    const float4* slab;   // null: plain range
    int splits, G, blk0, pad;
};
struct SlabRanges {
    int n;
    SlabRange r[2 * FH_MAX_GRAD_SLABS + 1];
};
struct OptScal {  // SGD: neg_lr, mom, wd, first | Adam: the adam_elem scalars
    float neg_lr, mom, wd;
    int first;
    float decay_mul, one_m_b1, b2, one_m_b2, bc2_sqrt, eps, neg_step_size;
    int decoupled;
    const float* scal;  // Adam: device {bc2_sqrt, -step_size} or null
};

constexpr int kOptPlainPer = 1024;  // float4s per plain block

// DP-SGD (r04): the same launch finishes a per-sample-clipped step.  Slab ranges hold one
// split per IMAGE (conv.hip fh_conv2d_wgrad_persample): g = sum_{i < count} coef[z][i] *
// slab[z][i] in image order (fh_persample_slab_wsum's operations); then, on elements
// [0, n_noise) of the row, g += (sigma_c / count) * N(0,1) with fh_dpsgd_noise's Philox keys
// (key = seed + *seed_dev, row philox_row(seed_dev, z), counter = the row's float4 index) —
// the bits of slab_wsum + dpsgd_noise + the optimizer step, in one pass.
struct OptDp {
    const float* coef;  // [client][batch]
    const int32_t* counts;
    int batch;
    int64_t n_noise;
    float sigma_c;
    uint64_t seed;
    const uint64_t* seed_dev;
};

__device__ __forceinline__ void dp_noise4(float4& g, const OptDp& d, uint64_t key, uint64_t row,
                                          int64_t q, float s) {
    if (s == 0.f) return;
    float r[4];
    gauss4(key, row, (uint64_t)q, r);
    const int64_t j = 4 * q;
    if (j < d.n_noise) g.x = g.x + s * r[0];
    if (j + 1 < d.n_noise) g.y = g.y + s * r[1];
    if (j + 2 < d.n_noise) g.z = g.z + s * r[2];
    if (j + 3 < d.n_noise) g.w = g.w + s * r[3];
}

// The update of one float4 in two phases: opt_load4 issues its loads (p and the state, from
// in-bounds addresses — a missing momentum buffer reads p — so no load sits under a branch),
// opt_apply4 computes and stores.  The plain ranges load all their float4s first (r05: with
// the momentum load under `if (use_buf)` each float4's loads and update were one dependent
// round trip).
struct OptIn {
    float4 p, m, v;
};
template <bool ADAM>
__device__ __forceinline__ void opt_load4(const float4* p, const float4* s1, const float4* s2,
                                          int64_t i, OptIn& in) {
    in.p = p[i];
    in.m = (s1 ? s1 : p)[i];
    if constexpr (ADAM) in.v = s2[i];
}

template <bool ADAM>
__device__ __forceinline__ void opt_apply4(float4* p, float4* s1, float4* s2, int64_t i,
                                           const OptIn& in, float4 gv, const OptScal& o,
                                           float bc2_sqrt, float neg_step) {
    const float4 pv = in.p;
    float4 out;
    if constexpr (!ADAM) {
        const bool use_buf = o.mom != 0.f;
        const float4 bv = (use_buf && !o.first) ? in.m : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 b;
        out.x = sgd_elem(pv.x, gv.x, bv.x, o.neg_lr, o.mom, o.wd, o.first, b.x);
        out.y = sgd_elem(pv.y, gv.y, bv.y, o.neg_lr, o.mom, o.wd, o.first, b.y);
        out.z = sgd_elem(pv.z, gv.z, bv.z, o.neg_lr, o.mom, o.wd, o.first, b.z);
        out.w = sgd_elem(pv.w, gv.w, bv.w, o.neg_lr, o.mom, o.wd, o.first, b.w);
        if (use_buf) s1[i] = b;
    } else {
        float4 mv = in.m, vv = in.v;
#define FH_ADAM_LANE(c) out.c = adam_elem(pv.c, gv.c, mv.c, vv.c, o.wd, o.decay_mul, o.decoupled, \
                                          o.one_m_b1, o.b2, o.one_m_b2, bc2_sqrt, o.eps, neg_step)
        FH_ADAM_LANE(x); FH_ADAM_LANE(y); FH_ADAM_LANE(z); FH_ADAM_LANE(w);
#undef FH_ADAM_LANE
        s1[i] = mv;
        s2[i] = vv;
    }
    p[i] = out;
}

template <bool ADAM, bool DP = false>
__global__ void __launch_bounds__(256)
opt_slabs_kernel(float4* __restrict__ p, float4* __restrict__ g, float4* __restrict__ s1,
                 float4* __restrict__ s2, int64_t row4, const SlabRanges rg, const OptScal o,
                 const OptDp d) {
    __shared__ float4 red[256];
    const int z = blockIdx.y, bx = blockIdx.x, t = threadIdx.x;
    int k = 0;
    for (int i = 1; i < rg.n; ++i)
        if (rg.r[i].blk0 <= bx) k = i;
    const SlabRange R = rg.r[k];
    const int64_t base = (int64_t)z * row4 + R.off4;
    const float bc2_sqrt = (ADAM && o.scal) ? o.scal[0] : o.bc2_sqrt;
    const float neg_step = (ADAM && o.scal) ? o.scal[1] : o.neg_step_size;
    if constexpr (DP) {
        const int cnt = d.counts ? d.counts[z] : d.batch;
        const float s = cnt > 0 ? d.sigma_c / (float)cnt : 0.f;
        const uint64_t key = d.seed + (d.seed_dev ? *d.seed_dev : 0ull);
        const uint64_t row = philox_row(d.seed_dev, z);
        if (R.slab == nullptr) {
            constexpr int U = kOptPlainPer / 256;
            const int i0 = (bx - R.blk0) * kOptPlainPer + t;
            OptIn in[U];
            float4 gq[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {  // every float4's loads first (as the plain path below)
                const int i = i0 + 256 * u < R.len4 ? i0 + 256 * u : 0;
                gq[u] = g[base + i];
                opt_load4<ADAM>(p, s1, s2, base + i, in[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + 256 * u;
                if (i < R.len4) {
                    float4 gv = gq[u];
                    dp_noise4(gv, d, key, row, (int64_t)R.off4 + i, s);
                    g[base + i] = gv;
                    opt_apply4<ADAM>(p, s1, s2, base + i, in[u], gv, o, bc2_sqrt, neg_step);
                }
            }
            return;
        }
        const int e = (bx - R.blk0) * 256 + t;
        if (e >= R.len4) return;
        OptIn in;  // the parameter / state loads in flight with the slab sums
        opt_load4<ADAM>(p, s1, s2, base + e, in);
        const float4* src = R.slab + (int64_t)z * R.splits * R.len4 + e;
        const float* cz = d.coef + (int64_t)z * d.batch;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        // fh_persample_slab_wsum's order and operations, eight images' loads in flight (r05:
        // one image at a time left one dependent round trip per image)
        for (int i0 = 0; i0 < cnt; i0 += 8) {
            float c[8];
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool ok = i0 + j < cnt;
                c[j] = ok ? cz[i0 + j] : 0.f;
                v[j] = ok ? src[(int64_t)(i0 + j) * R.len4] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j < cnt) {
                    acc.x = acc.x + c[j] * v[j].x;
                    acc.y = acc.y + c[j] * v[j].y;
                    acc.z = acc.z + c[j] * v[j].z;
                    acc.w = acc.w + c[j] * v[j].w;
                }
        }
        dp_noise4(acc, d, key, row, (int64_t)R.off4 + e, s);
        g[base + e] = acc;
        opt_apply4<ADAM>(p, s1, s2, base + e, in, acc, o, bc2_sqrt, neg_step);
        return;
    }
    if (R.slab == nullptr) {
        constexpr int U = kOptPlainPer / 256;
        const int i0 = (bx - R.blk0) * kOptPlainPer + t;
        OptIn in[U];
        float4 gq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every float4's loads first (past the range: its start)
            const int i = i0 + 256 * u < R.len4 ? i0 + 256 * u : 0;
            gq[u] = g[base + i];
            opt_load4<ADAM>(p, s1, s2, base + i, in[u]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + 256 * u;
            if (i < R.len4) opt_apply4<ADAM>(p, s1, s2, base + i, in[u], gq[u], o, bc2_sqrt, neg_step);
        }
        return;
    }
    const int G = R.G, C = 256 / G;
    const int e = (bx - R.blk0) * C + t % C;
    const int piece = t / C, splits = R.splits;
    const int s0 = (int)((int64_t)splits * piece / G), s1e = (int)((int64_t)splits * (piece + 1) / G);
    OptIn in;  // the updating thread's parameter / state loads in flight with the slab sums
    if (piece == 0) opt_load4<ADAM>(p, s1, s2, base + (e < R.len4 ? e : 0), in);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < R.len4) {
        const float4* src = R.slab + (int64_t)z * splits * R.len4 + e;
        for (int i0 = s0; i0 < s1e; i0 += 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                v[j] = i0 + j < s1e ? src[(int64_t)(i0 + j) * R.len4] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j < s1e) {
                    acc.x += v[j].x;
                    acc.y += v[j].y;
                    acc.z += v[j].z;
                    acc.w += v[j].w;
                }
        }
    }
    if (G > 1) {  // block-uniform
        red[t] = acc;
        __syncthreads();
        if (piece != 0) return;
        for (int q = 1; q < G; ++q) {
            const float4 w = red[t + C * q];
            acc.x += w.x;
            acc.y += w.y;
            acc.z += w.z;
            acc.w += w.w;
        }
    }
    if (e >= R.len4) return;
    g[base + e] = acc;
    opt_apply4<ADAM>(p, s1, s2, base + e, in, acc, o, bc2_sqrt, neg_step);
}

// conv.hip splitk_sum's thread-group count for a split count (kept identical: same bits)
static int slab_groups(int splits) {
    int G = 1;
    while (G < 16 && splits >= 16 * G) G *= 2;
    return G;
}

// host: the ranges of a row (slab ranges + the plain gaps) and their block offsets
static int build_ranges(const fh_grad_slab* slabs, int nslabs, int64_t row_len, SlabRanges& rg,
                        int& blocks, bool per_image = false) {
    FH_REQUIRE(nslabs >= 0 && nslabs <= FH_MAX_GRAD_SLABS, "step_slabs: %d slab ranges (max %d)",
               nslabs, FH_MAX_GRAD_SLABS);
    FH_REQUIRE(nslabs == 0 || slabs, "step_slabs: null slab array");
    FH_REQUIRE(row_len % 4 == 0 && row_len / 4 < (1ll << 30), "step_slabs: row_len %lld",
               (long long)row_len);
    rg.n = 0;
    blocks = 0;
    int64_t pos = 0;
    auto add = [&](int64_t off, int64_t len, const float* slab, int splits) {
        SlabRange& r = rg.r[rg.n++];
        r.off4 = (int)(off / 4);
        r.len4 = (int)(len / 4);
        r.slab = (const float4*)slab;
        r.splits = splits;
        r.G = (slab && !per_image) ? slab_groups(splits) : 1;
        r.blk0 = blocks;
        r.pad = 0;
        blocks += (int)(slab ? ceil_div(r.len4, 256 / r.G) : ceil_div(r.len4, kOptPlainPer));
    };
    for (int i = 0; i < nslabs; ++i) {
        const fh_grad_slab& s = slabs[i];
        FH_REQUIRE(s.off >= pos && s.len > 0 && s.off + s.len <= row_len && s.off % 4 == 0 &&
                       s.len % 4 == 0 && s.slab && (uintptr_t)s.slab % 16 == 0 && s.splits >= 1,
                   "step_slabs: bad slab range %d (off %lld len %lld splits %d)", i,
                   (long long)s.off, (long long)s.len, s.splits);
        if (s.off > pos) add(pos, s.off - pos, nullptr, 0);
        add(s.off, s.len, s.slab, s.splits);
        pos = s.off + s.len;
    }
    if (pos < row_len) add(pos, row_len - pos, nullptr, 0);
    return FH_OK;
}

}  // namespace fh

using namespace fh;

static int grid_for(int64_t n) { return (int)std::min<int64_t>(ceil_div(n, 256), 4096); }

extern "C" int fh_sgd_step_slabs(float* param, float* grad, float* momentum_buf,
                                 int64_t row_stride, int64_t row_len, int32_t nclients,
                                 const fh_grad_slab* slabs, int32_t nslabs, float lr,
                                 float momentum, float weight_decay, int32_t first_step,
                                 void* stream) {
    FH_REQUIRE(nclients >= 0 && row_stride >= row_len && row_stride % 4 == 0,
               "sgd_step_slabs: bad shape");
    if (nclients == 0 || row_len == 0) return FH_OK;
    FH_REQUIRE(param && grad && (momentum == 0.f || momentum_buf), "sgd_step_slabs: null pointer");
    FH_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)momentum_buf) % 16 == 0,
               "sgd_step_slabs: rows must be 16-B aligned");
    SlabRanges rg;
    int blocks = 0;
    if (const int rc = build_ranges(slabs, nslabs, row_len, rg, blocks)) return rc;
    OptScal o{};
    o.neg_lr = -lr;
    o.mom = momentum;
    o.wd = weight_decay;
    o.first = first_step;
    FH_LAUNCH(opt_slabs_kernel<false>, dim3(blocks, nclients), dim3(256), 0, as_stream(stream),
              (float4*)param, (float4*)grad, (float4*)momentum_buf, (float4*)nullptr,
              row_stride / 4, rg, o, OptDp{});
    FH_LAUNCH_CHECK("sgd_step_slabs");
    return FH_OK;
}

extern "C" int fh_adam_step_slabs(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                                  int64_t row_stride, int64_t row_len, int32_t nclients,
                                  const fh_grad_slab* slabs, int32_t nslabs, double lr,
                                  double beta1, double beta2, double eps, double weight_decay,
                                  int32_t decoupled, double step_size, double bc2_sqrt,
                                  const float* scal_dev, void* stream) {
    FH_REQUIRE(nclients >= 0 && row_stride >= row_len && row_stride % 4 == 0,
               "adam_step_slabs: bad shape");
    if (nclients == 0 || row_len == 0) return FH_OK;
    FH_REQUIRE(param && grad && exp_avg && exp_avg_sq, "adam_step_slabs: null pointer");
    FH_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) %
                       16 == 0,
               "adam_step_slabs: rows must be 16-B aligned");
    SlabRanges rg;
    int blocks = 0;
    if (const int rc = build_ranges(slabs, nslabs, row_len, rg, blocks)) return rc;
    // fh_adam_step's fp32 roundings of the double scalars
    OptScal o{};
    o.wd = (float)weight_decay;
    o.decay_mul = (float)(1.0 - lr * weight_decay);
    o.decoupled = decoupled;
    o.one_m_b1 = (float)(1.0 - beta1);
    o.b2 = (float)beta2;
    o.one_m_b2 = (float)(1.0 - beta2);
    o.bc2_sqrt = (float)bc2_sqrt;
    o.eps = (float)eps;
    o.neg_step_size = (float)(-step_size);
    o.scal = scal_dev;
    FH_LAUNCH(opt_slabs_kernel<true>, dim3(blocks, nclients), dim3(256), 0, as_stream(stream),
              (float4*)param, (float4*)grad, (float4*)exp_avg, (float4*)exp_avg_sq,
              row_stride / 4, rg, o, OptDp{});
    FH_LAUNCH_CHECK("adam_step_slabs");
    return FH_OK;
}

extern "C" int fh_dpsgd_step_slabs(float* param, float* grad, float* state1, float* state2,
                                   int64_t row_stride, int64_t row_len, int32_t nclients,
                                   const fh_grad_slab* slabs, int32_t nslabs, const float* coef,
                                   const int32_t* counts, int32_t batch, int64_t n_noise,
                                   float sigma_c, uint64_t seed, const uint64_t* seed_dev,
                                   int32_t adam, double lr, double momentum, double beta1,
                                   double beta2, double eps, double weight_decay,
                                   int32_t decoupled, int32_t first_step, double step_size,
                                   double bc2_sqrt, const float* scal_dev, void* stream) {
    FH_REQUIRE(nclients >= 0 && row_stride >= row_len && row_stride % 4 == 0 && batch > 0 &&
                   n_noise >= 0 && n_noise <= row_len && sigma_c >= 0.f,
               "dpsgd_step_slabs: bad shape");
    if (nclients == 0 || row_len == 0) return FH_OK;
    FH_REQUIRE(param && grad && coef && state1 && (!adam || state2),
               "dpsgd_step_slabs: null pointer");
    FH_REQUIRE(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)state1 |
                (adam ? (uintptr_t)state2 : 0)) % 16 == 0,
               "dpsgd_step_slabs: rows must be 16-B aligned");
    for (int i = 0; i < nslabs; ++i)
        FH_REQUIRE(slabs[i].splits == batch, "dpsgd_step_slabs: slab %d has %d splits, not one "
                   "per image (%d)", i, slabs[i].splits, batch);
    SlabRanges rg;
    int blocks = 0;
    if (const int rc = build_ranges(slabs, nslabs, row_len, rg, blocks, true)) return rc;
    OptScal o{};
    OptDp d{coef, counts, batch, n_noise, sigma_c, seed, seed_dev};
    hipStream_t st = as_stream(stream);
    if (!adam) {
        o.neg_lr = (float)-lr;
        o.mom = (float)momentum;
        o.wd = (float)weight_decay;
        o.first = first_step;
        FH_LAUNCH((opt_slabs_kernel<false, true>), dim3(blocks, nclients), dim3(256), 0, st,
                  (float4*)param, (float4*)grad, (float4*)state1, (float4*)nullptr,
                  row_stride / 4, rg, o, d);
    } else {
        o.wd = (float)weight_decay;
        o.decay_mul = (float)(1.0 - lr * weight_decay);
        o.decoupled = decoupled;
        o.one_m_b1 = (float)(1.0 - beta1);
        o.b2 = (float)beta2;
        o.one_m_b2 = (float)(1.0 - beta2);
        o.bc2_sqrt = (float)bc2_sqrt;
        o.eps = (float)eps;
        o.neg_step_size = (float)(-step_size);
        o.scal = scal_dev;
        FH_LAUNCH((opt_slabs_kernel<true, true>), dim3(blocks, nclients), dim3(256), 0, st,
                  (float4*)param, (float4*)grad, (float4*)state1, (float4*)state2,
                  row_stride / 4, rg, o, d);
    }
    FH_LAUNCH_CHECK("dpsgd_step_slabs");
    return FH_OK;
}

extern "C" int fh_sgd_step(float* param, const float* grad, float* momentum_buf, int64_t n,
                           float lr, float momentum, float weight_decay, int32_t first_step,
                           void* stream) {
    FH_REQUIRE(n >= 0, "sgd_step: bad size");
    if (n == 0) return FH_OK;
    FH_REQUIRE(param && grad && (momentum == 0.f || momentum_buf), "sgd_step: null pointer");
    const bool vec = n % 4 == 0 && ((uintptr_t)param | (uintptr_t)grad |
                                    (momentum != 0.f ? (uintptr_t)momentum_buf : 0)) % 16 == 0;
    if (vec)
        FH_LAUNCH(sgd4_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream),
                           (float4*)param, (const float4*)grad, (float4*)momentum_buf, n / 4, -lr,
                           momentum, weight_decay, first_step);
    else
        FH_LAUNCH(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), param,
                           grad, momentum_buf, n, -lr, momentum, weight_decay, first_step);
    FH_LAUNCH_CHECK("sgd_step");
    return FH_OK;
}

extern "C" int fh_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                            int64_t n, double lr, double beta1, double beta2, double eps,
                            double weight_decay, int32_t decoupled, double step_size,
                            double bc2_sqrt, const float* scal_dev, void* stream) {
    FH_REQUIRE(n >= 0, "adam_step: bad size");
    if (n == 0) return FH_OK;
    FH_REQUIRE(param && grad && exp_avg && exp_avg_sq, "adam_step: null pointer");
    // Python-double scalars are rounded to fp32 where ATen meets the fp32 tensor.
    const bool vec = n % 4 == 0 &&
                     ((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) %
                             16 == 0;
    if (vec)
        FH_LAUNCH(adam4_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream),
                           (float4*)param, (const float4*)grad, (float4*)exp_avg,
                           (float4*)exp_avg_sq, n / 4, (float)weight_decay,
                           (float)(1.0 - lr * weight_decay), decoupled, (float)(1.0 - beta1),
                           (float)beta2, (float)(1.0 - beta2), (float)bc2_sqrt, (float)eps,
                           (float)(-step_size), scal_dev);
    else
        FH_LAUNCH(adam_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), param,
                           grad, exp_avg, exp_avg_sq, n, (float)weight_decay,
                           (float)(1.0 - lr * weight_decay), decoupled, (float)(1.0 - beta1),
                           (float)beta2, (float)(1.0 - beta2), (float)bc2_sqrt, (float)eps,
                           (float)(-step_size), scal_dev);
    FH_LAUNCH_CHECK("adam_step");
    return FH_OK;
}
