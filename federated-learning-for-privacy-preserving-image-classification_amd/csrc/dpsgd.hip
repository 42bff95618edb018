// dpsgd.hip — per-sample-clipped DP-SGD (north_star "per-sample gradient clipping"; the
// reference clips whole-update deltas only, privacy.py:107-144).  Per optimizer step:
//
//   g_i  = grad of sample i's own loss  (the kernels hold g_i / B: CE is a batch mean)
//   c_i  = min(1, C / ||g_i||)           ||g_i||^2 summed over every parameter tensor
//   g    = (sum_i c_i g_i + sigma * C * xi) / B,   xi ~ N(0, I)  (Philox4x32-10)
//
// sigma defaults to the reference's Gaussian-mechanism multiplier sqrt(2 ln(1.25/delta))/eps
// (privacy.py:209).  Norms: conv layers via per-image WGRAD tiles (conv.hip,
// fh_conv2d_persample_sqnorm), linear layers via the rank-1 identity
// ||dy_i x_i^T||^2 = ||dy_i||^2 ||x_i||^2 (+ ||dy_i||^2 for the bias).  The clipped sum
// is the ordinary WGRAD run on dY rows pre-scaled by c_i (fh_scale_rows).
#include "fh_common.h"

namespace fh {

// sqnorm[z][i] += (||dy_i||^2 (||x_i||^2 + with_bias)) for i < cnt_z.  One block per (z, i).
__global__ void __launch_bounds__(256)
linear_sq_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ dy,
                 int64_t dy_cs, int with_bias, const int32_t* __restrict__ counts, int batch,
                 int in_f, int out_f, double* __restrict__ sqnorm) {
    __shared__ double red[4];
    const int i = blockIdx.x, z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    if (i >= cnt) return;  // block-uniform
    const float* xr = x + z * x_cs + (int64_t)i * in_f;
    const float* dr = dy + z * dy_cs + (int64_t)i * out_f;
    double sx = 0.0, sd = 0.0;
    for (int k = threadIdx.x; k < in_f; k += 256) sx += (double)xr[k] * (double)xr[k];
    for (int k = threadIdx.x; k < out_f; k += 256) sd += (double)dr[k] * (double)dr[k];
    sx = block_sum_256(sx, red);
    sd = block_sum_256(sd, red);
    if (threadIdx.x == 0) sqnorm[(int64_t)z * batch + i] += sd * (sx + (with_bias ? 1.0 : 0.0));
}

__global__ void __launch_bounds__(256)
clip_coef_kernel(const double* __restrict__ sqnorm, const int32_t* __restrict__ counts,
                 int nclients, int batch, double max_norm, float* __restrict__ coef) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= nclients * batch) return;
    const int z = e / batch, i = e - z * batch;
    const int cnt = counts ? counts[z] : batch;
    float c = 0.f;
    if (i < cnt) {
        // ||g_i|| = B * ||g_i / B||  (the stored gradients are of the batch-mean loss)
        const double norm = (double)cnt * sqrt(sqnorm[e]);
        c = norm > max_norm ? (float)(max_norm / norm) : 1.0f;
    }
    coef[e] = c;
}

// out[z][i][:] = coef[z][i] * in[z][i][:]  (rows of per_img floats; rows >= cnt -> 0)
__global__ void __launch_bounds__(256)
scale_rows_kernel(const float* __restrict__ in, int64_t in_cs, const float* __restrict__ coef,
                  const int32_t* __restrict__ counts, int batch, int64_t per_img,
                  float* __restrict__ out, int64_t out_cs) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    const int64_t total = (int64_t)batch * per_img;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(e / per_img);
        out[z * out_cs + e] = i < cnt ? coef[(int64_t)z * batch + i] * in[z * in_cs + e] : 0.f;
    }
}

// grad[z][j] += (sigma*C / cnt_z) * N(0,1), j < n; Philox keyed (seed, z, j/4)
__global__ void __launch_bounds__(256)
dpsgd_noise_kernel(float* __restrict__ grad, int64_t g_cs, int64_t n,
                   const int32_t* __restrict__ counts, int batch, float sigma_c, uint64_t seed,
                   const uint64_t* __restrict__ seed_dev) {
    const int z = blockIdx.y;
    const int cnt = counts ? counts[z] : batch;
    if (cnt <= 0) return;
    const uint64_t key = seed + (seed_dev ? *seed_dev : 0ull);
    const float s = sigma_c / (float)cnt;
    float* g = grad + z * g_cs;
    const int64_t nq = (n + 3) / 4;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nq;
         q += (int64_t)gridDim.x * blockDim.x) {
        float r[4];
        gauss4(key, philox_row(seed_dev, z), (uint64_t)q, r);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t j = q * 4 + u;
            if (j < n) g[j] = g[j] + s * r[u];
        }
    }
}

static unsigned ew_blocks(int64_t n) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), 2048));
}

}  // namespace fh

using namespace fh;

extern "C" int fh_linear_persample_sqnorm(const float* x, int64_t x_cs, const float* dy,
                                          int64_t dy_cs, int32_t with_bias, double* sqnorm,
                                          const int32_t* counts, int32_t nclients, int32_t batch,
                                          int32_t in_f, int32_t out_f, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && in_f > 0 && out_f > 0, "linear_persample_sqnorm: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && dy && sqnorm, "linear_persample_sqnorm: null pointer");
    FH_LAUNCH(linear_sq_kernel, dim3(batch, nclients), dim3(256), 0, as_stream(stream), x,
                       x_cs, dy, dy_cs, with_bias, counts, batch, in_f, out_f, sqnorm);
    FH_LAUNCH_CHECK("linear_persample_sqnorm");
    return FH_OK;
}

extern "C" int fh_dpsgd_clip_coef(const double* sqnorm, const int32_t* counts, int32_t nclients,
                                  int32_t batch, double max_norm, float* coef, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0, "dpsgd_clip_coef: bad shape");
    FH_REQUIRE(max_norm > 0.0, "dpsgd_clip_coef: max_norm must be > 0");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(sqnorm && coef, "dpsgd_clip_coef: null pointer");
    const int n = nclients * batch;
    FH_LAUNCH(clip_coef_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                       as_stream(stream), sqnorm, counts, nclients, batch, max_norm, coef);
    FH_LAUNCH_CHECK("dpsgd_clip_coef");
    return FH_OK;
}

extern "C" int fh_scale_rows(const float* in, int64_t in_cs, const float* coef,
                             const int32_t* counts, int32_t nclients, int32_t batch,
                             int64_t per_img, float* out, int64_t out_cs, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && per_img > 0, "scale_rows: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(in && coef && out, "scale_rows: null pointer");
    FH_LAUNCH(scale_rows_kernel, dim3(ew_blocks((int64_t)batch * per_img), nclients),
                       dim3(256), 0, as_stream(stream), in, in_cs, coef, counts, batch, per_img,
                       out, out_cs);
    FH_LAUNCH_CHECK("scale_rows");
    return FH_OK;
}

extern "C" int fh_dpsgd_noise(float* grad, int64_t g_cs, int64_t n, const int32_t* counts,
                              int32_t nclients, int32_t batch, float sigma_c, uint64_t seed,
                              const uint64_t* seed_dev, void* stream) {
    FH_REQUIRE(nclients >= 0 && batch > 0 && n >= 0, "dpsgd_noise: bad shape");
    FH_REQUIRE(sigma_c >= 0.f, "dpsgd_noise: sigma*C must be >= 0");
    if (nclients == 0 || n == 0 || sigma_c == 0.f) return FH_OK;
    FH_REQUIRE(grad, "dpsgd_noise: null pointer");
    FH_LAUNCH(dpsgd_noise_kernel, dim3(ew_blocks(ceil_div(n, 4)), nclients), dim3(256), 0,
                       as_stream(stream), grad, g_cs, n, counts, batch, sigma_c, seed, seed_dev);
    FH_LAUNCH_CHECK("dpsgd_noise");
    return FH_OK;
}
