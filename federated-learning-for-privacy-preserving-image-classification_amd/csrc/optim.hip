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

}  // namespace fh

using namespace fh;

static int grid_for(int64_t n) { return (int)std::min<int64_t>(ceil_div(n, 256), 4096); }

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
