// fh_common.h — shared definitions for libfedhip (gfx950 / CDNA4 only).
//
// Build contract (see build_native.py): every TU is compiled with
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
// so no multiply-add is ever contracted behind our back; every fused
// multiply-add in this library is an explicit fmaf() placed where the CPU
// reference (ATen's vectorised kernels) also fuses.  That is what keeps
// FedAvg bit-exact (reference fedavg.py:278-285 is mul-round-then-add-round).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <string>
#include <tuple>
#include <type_traits>
#include <utility>

#include "../../include/fedhip.h"

namespace fh {

// ---- error plumbing --------------------------------------------------------
void set_error(const char* fmt, ...);

#define FH_REQUIRE(cond, ...)                                   \
    do {                                                        \
        if (!(cond)) {                                          \
            ::fh::set_error(__VA_ARGS__);                       \
            return FH_E_INVALID;                                \
        }                                                       \
    } while (0)

#define FH_LAUNCH_CHECK(name)                                          \
    do {                                                               \
        hipError_t _e = hipGetLastError();                             \
        if (_e != hipSuccess) {                                        \
            ::fh::set_error("%s: launch failed: %s", name,             \
                            hipGetErrorString(_e));                    \
            return FH_E_LAUNCH;                                        \
        }                                                              \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- kernel launches -------------------------------------------------------
// Every kernel of the library is launched through FH_LAUNCH: the arguments are packed
// into an owned, typed tuple (the kernel's own parameter types) and issued with
// hipLaunchKernel.  While a step program is being recorded on this thread (program.hip,
// fh_record_begin) the launch is also appended to it with its own copy of the argument
// bytes, so a program never borrows storage from a HIP graph or the runtime.  The launch
// geometry is validated before anything reaches the queue (an empty grid would be a
// malformed dispatch packet).
struct KernelArgs {
    virtual ~KernelArgs() = default;
    void** params = nullptr;
    const size_t* sizes = nullptr;  // bytes of each argument (program relocation, program.hip)
    int nargs = 0;
};

template <typename... P>
struct KernelArgsT final : KernelArgs {
    std::tuple<P...> vals;
    void* ptrs[sizeof...(P) > 0 ? sizeof...(P) : 1];
    size_t szs[sizeof...(P) > 0 ? sizeof...(P) : 1];
    explicit KernelArgsT(P... p) : vals(p...) { bind(std::index_sequence_for<P...>{}); }
    KernelArgsT(const KernelArgsT&) = delete;
    KernelArgsT& operator=(const KernelArgsT&) = delete;

   private:
    template <size_t... I>
    void bind(std::index_sequence<I...>) {
        ((ptrs[I] = (void*)&std::get<I>(vals)), ...);
        ((szs[I] = sizeof(std::tuple_element_t<I, std::tuple<P...>>)), ...);
        params = ptrs;
        sizes = szs;
        nargs = (int)sizeof...(P);
    }
};

struct Recorder;                            // program.hip
extern thread_local Recorder* g_recorder;   // non-null while recording a step program
void record_kernel(Recorder* r, const void* func, dim3 grid, dim3 block, size_t shmem,
                   KernelArgs* args /* ownership passes */);

inline bool launch_geometry_ok(dim3 grid, dim3 block) {
    return grid.x && grid.y && grid.z && block.x && block.y && block.z &&
           block.x * block.y * block.z <= 1024 && grid.y <= 65535u && grid.z <= 65535u;
}

template <typename... P, typename... A>
inline hipError_t launch_kernel(void (*k)(P...), dim3 grid, dim3 block, size_t shmem,
                                hipStream_t st, A&&... a) {
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    if (!launch_geometry_ok(grid, block)) return hipErrorInvalidConfiguration;
    if (g_recorder) {
        auto* owned = new KernelArgsT<std::decay_t<P>...>(static_cast<std::decay_t<P>>(a)...);
        const hipError_t e = hipLaunchKernel((const void*)k, grid, block, owned->params, shmem, st);
        if (e != hipSuccess) {
            delete owned;
            return e;
        }
        record_kernel(g_recorder, (const void*)k, grid, block, shmem, owned);
        return e;
    }
    KernelArgsT<std::decay_t<P>...> args(static_cast<std::decay_t<P>>(a)...);
    return hipLaunchKernel((const void*)k, grid, block, args.params, shmem, st);
}

#define FH_LAUNCH(kernel, grid, block, shmem, stream, ...)                                  \
    do {                                                                                    \
        const hipError_t _le = ::fh::launch_kernel(kernel, grid, block, shmem, stream,      \
                                                   __VA_ARGS__);                            \
        if (_le != hipSuccess) {                                                            \
            ::fh::set_error("%s: launch of %s failed: %s", __func__, #kernel,               \
                            hipGetErrorString(_le));                                        \
            return FH_E_LAUNCH;                                                             \
        }                                                                                   \
    } while (0)

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---- fast unsigned division by a launch-constant divisor ------------------
// Round-up magic multiplier (Granlund–Montgomery); exact for n < 2^31.
struct FastDiv {
    uint32_t d, mul, shr;
    FastDiv() : d(1), mul(0), shr(0) {}
    explicit FastDiv(uint32_t div) : d(div) {
        shr = 0;
        while ((1u << shr) < div) ++shr;
        uint64_t one = 1;
        mul = (uint32_t)(((one << 32) * ((one << shr) - div)) / div + 1);
    }
    __host__ __device__ __forceinline__ uint32_t div(uint32_t n) const {
#ifdef __HIP_DEVICE_COMPILE__
        uint32_t t = __umulhi(n, mul);
#else
        uint32_t t = (uint32_t)(((uint64_t)n * mul) >> 32);
#endif
        return (t + n) >> shr;
    }
    __host__ __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const {
        q = div(n);
        r = n - q * d;
    }
};

// ---- wave helpers (wave64) ------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Block-wide double sum for blockDim.x == 256 (4 waves); result valid in all threads.
__device__ __forceinline__ double block_sum_256(double v, double* red /*[4]*/) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double r = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return r;
}

// ---- Philox4x32-10 counter RNG (dropout masks, DP noise) ------------------
struct Philox {
    __device__ __forceinline__ static uint4 round(uint4 c, uint2 k) {
        const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
        uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
        uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
        return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    }
    __device__ __forceinline__ static uint4 gen(uint64_t seed, uint64_t ctr_hi, uint64_t ctr_lo) {
        uint4 c = make_uint4((uint32_t)ctr_lo, (uint32_t)(ctr_lo >> 32),
                             (uint32_t)ctr_hi, (uint32_t)(ctr_hi >> 32));
        uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            c = round(c, k);
            k.x += 0x9E3779B9u;
            k.y += 0xBB67AE85u;
        }
        return c;
    }
};
// Philox row key of local row z.  seed_dev (nullable) points to the device key block
// {step key, n_ids, id[0..n_ids)}: with n_ids != 0 row z draws under its GLOBAL client id, so a
// client's dropout / augmentation / DP-SGD noise streams do not depend on the rank, lane or
// slot it trains in; else under z (callers then salt the seed per lane and rank).
__device__ __forceinline__ uint64_t philox_row(const uint64_t* seed_dev, int z) {
    return (seed_dev != nullptr && seed_dev[1] != 0ull) ? seed_dev[2 + z] : (uint64_t)z;
}

// uniform in (0, 1]
__device__ __forceinline__ float u01(uint32_t x) {
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// four N(0,1) draws (Box-Muller on one Philox block)
__device__ __forceinline__ void gauss4(uint64_t seed, uint64_t hi, uint64_t lo, float g[4]) {
    const uint4 r = Philox::gen(seed, hi, lo);
    const float ra = sqrtf(-2.0f * logf(u01(r.x))), rb = sqrtf(-2.0f * logf(u01(r.z)));
    float sa, ca, sb, cb;
    sincosf(6.2831853071795864f * u01(r.y), &sa, &ca);
    sincosf(6.2831853071795864f * u01(r.w), &sb, &cb);
    g[0] = ra * ca;
    g[1] = ra * sa;
    g[2] = rb * cb;
    g[3] = rb * sb;
}

}  // namespace fh
