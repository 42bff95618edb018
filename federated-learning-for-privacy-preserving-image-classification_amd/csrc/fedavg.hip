// fedavg.hip — FedAvg weighted reduction and update validation statistics.
//
// Reference: FedAvgAggregator._weighted_average, src/aggregation/fedavg.py:267-289:
//     aggregated[l] = zeros_like(ref[l])
//     for update, weight in zip(updates, weights):      # client-list order
//         aggregated[l] += weight * update.model_weights[l]
// `weight` is a Python float, rounded to fp32 when it multiplies the fp32
// tensor; the product is rounded, then the sum.  This kernel keeps exactly
// that rounding sequence (the TU is built with -ffp-contract=off, no fmaf
// here), so the aggregate is bit-identical to the reference on one GPU.
//
// HBM-bound: reads C*P floats, writes P.  Each thread owns 4 consecutive
// parameters (16-B loads/stores) and walks the clients in order, keeping
// four client rows in flight to cover HBM latency.
#include "fh_common.h"

namespace fh {

__global__ void __launch_bounds__(256)
fedavg_vec4_kernel(const float* __restrict__ rows, int64_t row_stride,
                   const int32_t* __restrict__ row_index, const float* __restrict__ weights, int C,
                   int64_t P4, float* __restrict__ out, int accumulate) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < P4;
         q += (int64_t)gridDim.x * blockDim.x) {
        float4 acc = accumulate ? reinterpret_cast<const float4*>(out)[q]
                                : make_float4(0.f, 0.f, 0.f, 0.f);
        int k = 0;
        for (; k + 4 <= C; k += 4) {
            float4 x[4];
            float w[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t r = row_index ? row_index[k + u] : (k + u);
                x[u] = reinterpret_cast<const float4*>(rows + r * row_stride)[q];
                w[u] = weights[k + u];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc.x = acc.x + w[u] * x[u].x;
                acc.y = acc.y + w[u] * x[u].y;
                acc.z = acc.z + w[u] * x[u].z;
                acc.w = acc.w + w[u] * x[u].w;
            }
        }
        for (; k < C; ++k) {
            const int64_t r = row_index ? row_index[k] : k;
            const float4 x = reinterpret_cast<const float4*>(rows + r * row_stride)[q];
            const float w = weights[k];
            acc.x = acc.x + w * x.x;
            acc.y = acc.y + w * x.y;
            acc.z = acc.z + w * x.z;
            acc.w = acc.w + w * x.w;
        }
        reinterpret_cast<float4*>(out)[q] = acc;
    }
}

__global__ void __launch_bounds__(256)
fedavg_scalar_kernel(const float* __restrict__ rows, int64_t row_stride,
                     const int32_t* __restrict__ row_index, const float* __restrict__ weights,
                     int C, int64_t begin, int64_t P, float* __restrict__ out, int accumulate) {
    for (int64_t j = begin + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < P;
         j += (int64_t)gridDim.x * blockDim.x) {
        float acc = accumulate ? out[j] : 0.f;
        for (int k = 0; k < C; ++k) {
            const int64_t r = row_index ? row_index[k] : k;
            acc = acc + weights[k] * rows[r * row_stride + j];
        }
        out[j] = acc;
    }
}

// Per (segment t, client z): max |w| and NaN/Inf flag over the segment.
__global__ void __launch_bounds__(256)
update_stats_kernel(const float* __restrict__ rows, int64_t row_stride,
                    const int64_t* __restrict__ seg_off, int nseg, float* __restrict__ absmax,
                    int32_t* __restrict__ nonfinite) {
    __shared__ float smax[4];
    __shared__ int sbad[4];
    const int t = blockIdx.x, z = blockIdx.y;
    const int64_t b = seg_off[t], e = seg_off[t + 1];
    const float* r = rows + z * row_stride;
    float m = 0.f;
    int bad = 0;
    for (int64_t j = b + threadIdx.x; j < e; j += 256) {
        const float v = r[j];
        if (!isfinite(v)) bad = 1;
        else m = fmaxf(m, fabsf(v));
    }
    m = wave_max(m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bad |= __shfl_xor(bad, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        smax[wid] = m;
        sbad[wid] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        absmax[z * nseg + t] = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
        nonfinite[z * nseg + t] = sbad[0] | sbad[1] | sbad[2] | sbad[3];
    }
}

}  // namespace fh

using namespace fh;

extern "C" int fh_fedavg_weighted_sum(const float* rows, int64_t row_stride,
                                      const int32_t* row_index, const float* weights,
                                      int32_t num_clients, int64_t P, float* out,
                                      int32_t accumulate, void* stream) {
    FH_REQUIRE(num_clients >= 0 && P >= 0, "fedavg: bad sizes C=%d P=%lld", num_clients,
               (long long)P);
    if (P == 0) return FH_OK;
    FH_REQUIRE(out && (num_clients == 0 || (rows && weights)), "fedavg: null pointer");
    hipStream_t st = as_stream(stream);
    // 16-B path over the 4-aligned prefix (packed rows are padded to a multiple of 64
    // floats by the engine), scalar kernel for the < 4-element tail.
    const bool vec_ok = (row_stride % 4 == 0) && (reinterpret_cast<uintptr_t>(rows) % 16 == 0) &&
                        (reinterpret_cast<uintptr_t>(out) % 16 == 0);
    int64_t done = 0;
    if (vec_ok && P >= 4) {
        const int64_t P4 = P / 4;
        const int grid = (int)std::min<int64_t>(ceil_div(P4, 256), 8192);
        FH_LAUNCH(fedavg_vec4_kernel, dim3(grid), dim3(256), 0, st, rows, row_stride,
                           row_index, weights, num_clients, P4, out, accumulate);
        FH_LAUNCH_CHECK("fedavg_vec4");
        done = P4 * 4;
    }
    if (done < P) {
        const int grid = (int)std::min<int64_t>(ceil_div(P - done, 256), 8192);
        FH_LAUNCH(fedavg_scalar_kernel, dim3(grid), dim3(256), 0, st, rows, row_stride,
                           row_index, weights, num_clients, done, P, out, accumulate);
        FH_LAUNCH_CHECK("fedavg_scalar");
    }
    return FH_OK;
}

extern "C" int fh_update_stats(const float* rows, int64_t row_stride, int32_t num_clients,
                               const int64_t* seg_offsets, int32_t nseg, float* seg_absmax,
                               int32_t* seg_nonfinite, void* stream) {
    FH_REQUIRE(num_clients >= 0 && nseg >= 0, "update_stats: bad sizes");
    if (num_clients == 0 || nseg == 0) return FH_OK;
    FH_REQUIRE(rows && seg_offsets && seg_absmax && seg_nonfinite, "update_stats: null pointer");
    FH_LAUNCH(update_stats_kernel, dim3(nseg, num_clients), dim3(256), 0,
                       as_stream(stream), rows, row_stride, seg_offsets, nseg, seg_absmax,
                       seg_nonfinite);
    FH_LAUNCH_CHECK("update_stats");
    return FH_OK;
}
