// dp.hip — update-level differential privacy: clip the client delta to a global
// L2 norm, add Gaussian noise, reconstitute the uploaded weights.
//
// Reference chain (all fp32 tensors, Python-double scalars):
//   src/client/federated_trainer.py:438-443   delta = w_local - w_global
//   src/shared/privacy.py:119-123             total = sqrt(sum_t float(norm(delta_t))**2)
//   src/shared/privacy.py:127-133             if total > C: delta_t * (C/total) else clone
//   src/shared/privacy.py:140, 209            sigma = min(total, C) * sqrt(2 ln(1.25/delta)) / eps
//   src/shared/privacy.py:212, 245            noisy_t = delta_t + normal(0, sigma)
//   src/client/federated_trainer.py:457       w = w_global + noisy
// Three HBM-bound passes over the packed [clients][P] rows; no host sync in
// between (clip decision and sigma are computed on the device).
#include "fh_common.h"

#include <cstdlib>

namespace fh {

// One block per (segment, client): fp64 sum of squares of the fp32 delta.  1024 threads and
// float4 loads over the 16-B aligned body of the segment (scalar head / tail): one segment can
// be the whole fc1 weight (SimpleCNN 401,408 elements), which a 256-thread scalar loop took
// 0.67 ms per client row to walk.
template <int kSqThreads>
__global__ void __launch_bounds__(kSqThreads)
dp_sqnorm_kernel(const float* __restrict__ local, int64_t ls, const float* __restrict__ global,
                 int64_t gs, const int64_t* __restrict__ seg_off, int nseg,
                 double* __restrict__ out) {
    __shared__ double red[kSqThreads / 64];
    const int t = blockIdx.x, z = blockIdx.y;
    const int64_t b = seg_off[t], e = seg_off[t + 1];
    const float* l = local + z * ls;
    const float* g = global ? global + z * gs : nullptr;
    const bool vec = ((uintptr_t)l % 16 == 0) && (!g || (uintptr_t)g % 16 == 0);
    const int64_t hb = vec ? min(e, (b + 3) & ~(int64_t)3) : e;  // scalar head [b, hb)
    const int64_t ve = vec ? max(hb, e & ~(int64_t)3) : e;        // float4 body [hb, ve)
    double s = 0.0;
    for (int64_t j = b + threadIdx.x; j < hb; j += kSqThreads) {
        const float d = g ? (l[j] - g[j]) : l[j];
        s += (double)d * (double)d;
    }
    for (int64_t q = hb / 4 + threadIdx.x; q < ve / 4; q += kSqThreads) {
        float4 d = reinterpret_cast<const float4*>(l)[q];
        if (g) {
            const float4 gv = reinterpret_cast<const float4*>(g)[q];
            d.x = d.x - gv.x; d.y = d.y - gv.y; d.z = d.z - gv.z; d.w = d.w - gv.w;
        }
        s += ((double)d.x * d.x + (double)d.y * d.y) + ((double)d.z * d.z + (double)d.w * d.w);
    }
    for (int64_t j = ve + threadIdx.x; j < e; j += kSqThreads) {  // scalar tail
        const float d = g ? (l[j] - g[j]) : l[j];
        s += (double)d * (double)d;
    }
    s = wave_sum(s);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double v = 0.0;
        for (int w = 0; w < kSqThreads / 64; ++w) v += red[w];  // wave order
        out[z * nseg + t] = v;
    }
}

__global__ void dp_coef_kernel(const double* __restrict__ sq, int C, int nseg, double max_norm,
                               double noise_scale, double* __restrict__ total_out,
                               float* __restrict__ coef, int32_t* __restrict__ clipped,
                               float* __restrict__ sigma) {
    const int z = blockIdx.x * blockDim.x + threadIdx.x;
    if (z >= C) return;
    double tot = 0.0;
    for (int t = 0; t < nseg; ++t) {
        // grad.norm().item(): an fp32 norm promoted to double, then squared.
        const double nt = (double)(float)sqrt(sq[z * nseg + t]);
        tot += nt * nt;
    }
    tot = sqrt(tot);
    if (total_out) total_out[z] = tot;
    const int cl = tot > max_norm;
    clipped[z] = cl;
    coef[z] = cl ? (float)(max_norm / tot) : 1.0f;
    const double sens = tot < max_norm ? tot : max_norm;
    sigma[z] = (float)(sens * noise_scale);
}

// out = [global +] ((clipped ? fl32(delta * coef) : delta) + noise)
__global__ void __launch_bounds__(256)
dp_apply_kernel(const float* __restrict__ local, int64_t ls, const float* __restrict__ global,
                int64_t gs, float* __restrict__ out, int64_t os, int64_t P,
                const float* __restrict__ coef, const int32_t* __restrict__ clipped,
                const float* __restrict__ sigma, const float* __restrict__ noise, int64_t ns,
                uint64_t seed, const int64_t* __restrict__ row_ids) {
    const int z = blockIdx.y;
    // Philox key: the row's global client id when given (ranks / lanes hold different
    // clients in the same local row z — the noise must never repeat across clients)
    const uint64_t key = row_ids ? (uint64_t)row_ids[z] : (uint64_t)z;
    const float* l = local + z * ls;
    const float* g = global ? global + z * gs : nullptr;
    float* o = out + z * os;
    const float* nz = noise ? noise + z * ns : nullptr;
    const int cl = clipped[z];
    const float cf = coef[z], sg = sigma[z];
    const int64_t nq = (P + 3) / 4;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq;
         q += (int64_t)gridDim.x * blockDim.x) {
        float gauss[4];
        if (!nz) {
            const uint4 r = Philox::gen(seed, key, (uint64_t)q);
            const float u1a = u01(r.x), u2a = u01(r.y), u1b = u01(r.z), u2b = u01(r.w);
            const float ra = sqrtf(-2.0f * logf(u1a)), rb = sqrtf(-2.0f * logf(u1b));
            float sa, ca, sb, cb;
            sincosf(6.2831853071795864f * u2a, &sa, &ca);
            sincosf(6.2831853071795864f * u2b, &sb, &cb);
            gauss[0] = ra * ca;
            gauss[1] = ra * sa;
            gauss[2] = rb * cb;
            gauss[3] = rb * sb;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t j = q * 4 + u;
            if (j >= P) break;
            const float gv = g ? g[j] : 0.f;
            float d = g ? (l[j] - gv) : l[j];
            if (cl) d = d * cf;
            const float n = nz ? nz[j] : sg * gauss[u];
            const float noisy = d + n;
            o[j] = g ? (gv + noisy) : noisy;
        }
    }
}

}  // namespace fh

using namespace fh;

extern "C" int fh_dp_delta_sqnorm(const float* local, int64_t local_stride, const float* global,
                                  int64_t global_stride, int32_t num_clients,
                                  const int64_t* seg_offsets, int32_t nseg, double* seg_sqnorm,
                                  void* stream) {
    FH_REQUIRE(num_clients >= 0 && nseg >= 0, "dp_delta_sqnorm: bad sizes");
    if (num_clients == 0 || nseg == 0) return FH_OK;
    FH_REQUIRE(local && seg_offsets && seg_sqnorm, "dp_delta_sqnorm: null pointer");
    // 1024 threads per (segment, client): r02 s3 measured the 256-thread block at 0.67 ms per
    // K2 round on SimpleCNN's fc1.weight segment alone
    FH_LAUNCH(dp_sqnorm_kernel<1024>, dim3(nseg, num_clients), dim3(1024), 0, as_stream(stream),
              local, local_stride, global, global_stride, seg_offsets, nseg, seg_sqnorm);
    FH_LAUNCH_CHECK("dp_delta_sqnorm");
    return FH_OK;
}

extern "C" int fh_dp_clip_coef(const double* seg_sqnorm, int32_t num_clients, int32_t nseg,
                               double max_norm, double epsilon, double delta, double* total_norm,
                               float* coef, int32_t* clipped, float* sigma, void* stream) {
    FH_REQUIRE(num_clients >= 0 && nseg >= 0, "dp_clip_coef: bad sizes");
    FH_REQUIRE(epsilon > 0 && delta > 0 && delta < 1 && max_norm > 0,
               "dp_clip_coef: invalid privacy parameters eps=%g delta=%g C=%g", epsilon, delta,
               max_norm);
    if (num_clients == 0) return FH_OK;
    FH_REQUIRE(seg_sqnorm && coef && clipped && sigma, "dp_clip_coef: null pointer");
    // Gaussian mechanism noise scale per unit sensitivity (privacy.py:209), in double.
    const double noise_scale = sqrt(2.0 * log(1.25 / delta)) / epsilon;
    FH_LAUNCH(dp_coef_kernel, dim3((unsigned)ceil_div(num_clients, 64)), dim3(64), 0,
                       as_stream(stream), seg_sqnorm, num_clients, nseg, max_norm, noise_scale,
                       total_norm, coef, clipped, sigma);
    FH_LAUNCH_CHECK("dp_clip_coef");
    return FH_OK;
}

extern "C" int fh_dp_apply(const float* local, int64_t local_stride, const float* global,
                           int64_t global_stride, float* out, int64_t out_stride,
                           int32_t num_clients, int64_t P, const float* coef,
                           const int32_t* clipped, const float* sigma, const float* noise_in,
                           int64_t noise_stride, uint64_t seed, const int64_t* row_ids,
                           void* stream) {
    FH_REQUIRE(num_clients >= 0 && P >= 0, "dp_apply: bad sizes");
    if (num_clients == 0 || P == 0) return FH_OK;
    FH_REQUIRE(local && out && coef && clipped && sigma, "dp_apply: null pointer");
    const int64_t nq = (P + 3) / 4;
    const int gx = (int)std::min<int64_t>(ceil_div(nq, 256), 2048);
    FH_LAUNCH(dp_apply_kernel, dim3(gx, num_clients), dim3(256), 0, as_stream(stream),
                       local, local_stride, global, global_stride, out, out_stride, P, coef,
                       clipped, sigma, noise_in, noise_stride, seed, row_ids);
    FH_LAUNCH_CHECK("dp_apply");
    return FH_OK;
}
