// compress.hip — update compression of packed client rows.
//
// Reference: src/shared/compression.py
//   QuantizationCompressor._quantize_tensor / _dequantize_tensor   :203-244
//   TopKSparsificationCompressor._sparsify_tensor / _desparsify_tensor :327-365
// applied per parameter tensor ("segment") of every client row.  What runs here is
// decompress(compress(v)) — the dense tensor the server would reconstruct — plus the
// wire codes (quantisation) or keep-mask (top-k), with v = x - base when a base row
// (the global model) is given, so the update delta is compressed and
// out = base + decompress(compress(x - base)).
//
// Work decomposition: every segment is cut into CHUNK-element chunks; the caller passes
// the cumulative chunk counts per segment (chunk_offsets[nseg+1]) and each workgroup of
// a (chunk, client) grid finds its segment by binary search.  Everything is HBM-bound
// byte work: no MFMA.
//
// Quantisation (2 launches): per-chunk min/max, then per element the segment's scale and
// zero point are recomputed from the chunk partials in the reference's double arithmetic
// (scale = 2*max|v| / (L-1) or (max-min)/(L-1), zp = (L-1)//2 or -round(min/scale)) and
// codes = clamp(rint(v / fl32(scale) + zp), 0, L-1), dense = (code - zp) * fl32(scale),
// all fp32 like ATen's CPU kernels.  Bit-exact with the reference (golden G8).
//
// Top-k by |v| (10 launches + a memset): MSB-first radix select over the 31-bit magnitude keys —
// four 8-bit histogram passes (LDS histograms, integer atomics: deterministic) each
// followed by a one-wave select that narrows the key prefix — gives the exact k-th
// largest key T and how many elements equal to T are kept; the apply pass keeps
// key > T and, among key == T, the lowest flat indices (documented tie rule: torch.topk
// leaves the order of equal magnitudes unspecified).
#include "fh_common.h"

namespace fh {

static constexpr int CQ_CHUNK = 8192;  // elements per workgroup (256 threads x 32)

__device__ __forceinline__ int seg_of_chunk(const int32_t* __restrict__ chunk_offsets,
                                            int nseg, int chunk) {
    int lo = 0, hi = nseg - 1;  // largest s with chunk_offsets[s] <= chunk
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (chunk_offsets[mid] <= chunk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ float delta_at(const float* __restrict__ x,
                                          const float* __restrict__ base, int64_t i) {
    return base ? x[i] - base[i] : x[i];
}

// ------------------------------------------------------------------ quantisation
__global__ void __launch_bounds__(256)
quant_minmax_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ base,
                    int64_t b_cs, const int64_t* __restrict__ seg_offsets,
                    const int32_t* __restrict__ chunk_offsets, int nseg, int nchunks,
                    float2* __restrict__ partial) {
    const int chunk = blockIdx.x, z = blockIdx.y;
    const int s = seg_of_chunk(chunk_offsets, nseg, chunk);
    const int64_t s0 = seg_offsets[s], s1 = seg_offsets[s + 1];
    const int64_t e0 = s0 + (int64_t)(chunk - chunk_offsets[s]) * CQ_CHUNK;
    const int64_t e1 = min(e0 + (int64_t)CQ_CHUNK, s1);
    const float* xr = x + z * x_cs;
    const float* br = base ? base + z * b_cs : nullptr;
    float mn = INFINITY, mx = -INFINITY;
    for (int64_t i = e0 + threadIdx.x; i < e1; i += 256) {
        const float v = delta_at(xr, br, i);
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
    __shared__ float smn[4], smx[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { smn[wid] = mn; smx[wid] = mx; }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[(int64_t)z * nchunks + chunk] =
            make_float2(fminf(fminf(smn[0], smn[1]), fminf(smn[2], smn[3])),
                        fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3])));
    }
}

__global__ void __launch_bounds__(256)
quant_apply_kernel(const float* x, int64_t x_cs, const float* __restrict__ base, int64_t b_cs,
                   float* out, int64_t o_cs, uint8_t* __restrict__ codes, int64_t c_cs,
                   const int64_t* __restrict__ seg_offsets,
                   const int32_t* __restrict__ chunk_offsets, int nseg, int nchunks,
                   const float2* __restrict__ partial, int levels, int symmetric,
                   double* __restrict__ scale_out, int64_t* __restrict__ zp_out) {
    const int chunk = blockIdx.x, z = blockIdx.y;
    const int s = seg_of_chunk(chunk_offsets, nseg, chunk);
    __shared__ double s_scale;
    __shared__ float s_zp;
    __shared__ int s_bad;
    if (threadIdx.x == 0) {
        float mn = INFINITY, mx = -INFINITY;
        for (int c = chunk_offsets[s]; c < chunk_offsets[s + 1]; ++c) {
            const float2 p = partial[(int64_t)z * nchunks + c];
            mn = fminf(mn, p.x);
            mx = fmaxf(mx, p.y);
        }
        double scale;
        int64_t zp;
        int bad = 0;
        if (symmetric) {
            const double max_val = (double)fmaxf(fabsf(mn), fabsf(mx));
            scale = (2.0 * max_val) / (double)(levels - 1);
            zp = (levels - 1) / 2;
        } else {
            scale = ((double)mx - (double)mn) / (double)(levels - 1);
            const double r = (double)mn / scale;
            // Python round() of +-inf / nan raises in the reference: flag, pass v through
            bad = !(scale > 0.0) || !isfinite(r);
            zp = bad ? 0 : -(int64_t)rint(r);
        }
        s_scale = scale;
        s_zp = (float)zp;
        s_bad = bad;
        if (chunk == chunk_offsets[s]) {  // one writer per (client, segment)
            if (scale_out) scale_out[(int64_t)z * nseg + s] = scale;
            if (zp_out) zp_out[(int64_t)z * nseg + s] = bad ? INT64_MIN : zp;
        }
    }
    __syncthreads();
    const float fs = (float)s_scale, fzp = s_zp, top = (float)(levels - 1);
    const int bad = s_bad;
    const int64_t s0 = seg_offsets[s], s1 = seg_offsets[s + 1];
    const int64_t e0 = s0 + (int64_t)(chunk - chunk_offsets[s]) * CQ_CHUNK;
    const int64_t e1 = min(e0 + (int64_t)CQ_CHUNK, s1);
    const float* xr = x + z * x_cs;
    const float* br = base ? base + z * b_cs : nullptr;
    float* orow = out ? out + z * o_cs : nullptr;
    uint8_t* crow = codes ? codes + z * c_cs : nullptr;
    for (int64_t i = e0 + threadIdx.x; i < e1; i += 256) {
        const float v = delta_at(xr, br, i);
        float q = rintf(__fdiv_rn(v, fs) + fzp);  // round half to even, as torch.round
        q = fminf(fmaxf(q, 0.f), top);             // NaN stays NaN (torch.clamp) ...
        if (q != q) q = 0.f;                        // ... and converts to code 0 on x86
        if (crow) crow[i] = (uint8_t)(int)q;
        if (orow) {
            const float d = bad ? v : (q - fzp) * fs;
            orow[i] = br ? br[i] + d : d;
        }
    }
}

// ------------------------------------------------------------------ top-k
struct TopkState {
    uint32_t prefix;  // key bits fixed so far
    uint32_t kr;      // rank still to place inside the prefix group (1-based)
    uint32_t cnt_eq;  // elements whose key == final threshold
    uint32_t pad;
};

__device__ __forceinline__ uint32_t mag_key(float v) {
    return __float_as_uint(v) & 0x7FFFFFFFu;  // |v| bits: monotonic in |v| (NaN on top)
}

__global__ void __launch_bounds__(256)
topk_hist_kernel(const float* __restrict__ x, int64_t x_cs, const float* __restrict__ base,
                 int64_t b_cs, const int64_t* __restrict__ seg_offsets,
                 const int32_t* __restrict__ chunk_offsets, int nseg,
                 const TopkState* __restrict__ state, uint32_t* __restrict__ hist, int round,
                 uint32_t* __restrict__ chunk_hist, int nchunks) {
    const int chunk = blockIdx.x, z = blockIdx.y;
    const int s = seg_of_chunk(chunk_offsets, nseg, chunk);
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    const int shift = 24 - 8 * round;
    const uint32_t mask = round == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    const uint32_t prefix = round == 0 ? 0u : state[(int64_t)z * nseg + s].prefix;
    __syncthreads();
    const int64_t s0 = seg_offsets[s], s1 = seg_offsets[s + 1];
    const int64_t e0 = s0 + (int64_t)(chunk - chunk_offsets[s]) * CQ_CHUNK;
    const int64_t e1 = min(e0 + (int64_t)CQ_CHUNK, s1);
    const float* xr = x + z * x_cs;
    const float* br = base ? base + z * b_cs : nullptr;
    for (int64_t i = e0 + threadIdx.x; i < e1; i += 256) {
        const uint32_t key = mag_key(delta_at(xr, br, i));
        if ((key & mask) == prefix) atomicAdd(&h[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t c = h[threadIdx.x];
    if (c) atomicAdd(&hist[((int64_t)z * nseg + s) * 256 + threadIdx.x], c);
    // last round: keep this chunk's histogram so the apply pass can rank ties at T by
    // index without re-reading (possibly already overwritten) earlier chunks
    if (chunk_hist) chunk_hist[((int64_t)z * nchunks + chunk) * 256 + threadIdx.x] = c;
}

__global__ void __launch_bounds__(64)
topk_select_kernel(const int64_t* __restrict__ seg_k, int nseg, TopkState* __restrict__ state,
                   uint32_t* __restrict__ hist, int round) {
    const int s = blockIdx.x, z = blockIdx.y;
    const int64_t sid = (int64_t)z * nseg + s;
    uint32_t* h = hist + sid * 256;
    if (threadIdx.x == 0) {
        TopkState st = state[sid];
        if (round == 0) { st.prefix = 0; st.kr = (uint32_t)seg_k[s]; }
        const int shift = 24 - 8 * round;
        uint32_t above = 0;
        int b = 255;
        for (; b > 0; --b) {
            if (above + h[b] >= st.kr) break;
            above += h[b];
        }
        st.prefix |= (uint32_t)b << shift;
        st.kr -= above;
        if (round == 3) st.cnt_eq = h[b];
        state[sid] = st;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) h[i] = 0;  // ready for the next round
}

__global__ void __launch_bounds__(256)
topk_apply_kernel(const float* x, int64_t x_cs, const float* __restrict__ base, int64_t b_cs,
                  float* out, int64_t o_cs, uint8_t* __restrict__ keep, int64_t k_cs,
                  const int64_t* __restrict__ seg_offsets,
                  const int32_t* __restrict__ chunk_offsets, int nseg,
                  const TopkState* __restrict__ state, const uint32_t* __restrict__ chunk_hist,
                  int nchunks) {
    const int chunk = blockIdx.x, z = blockIdx.y;
    const int s = seg_of_chunk(chunk_offsets, nseg, chunk);
    const TopkState st = state[(int64_t)z * nseg + s];
    const uint32_t T = st.prefix;
    const bool ranked = st.kr < st.cnt_eq;  // the tie at T is cut: keep the lowest indices
    const int64_t s0 = seg_offsets[s], s1 = seg_offsets[s + 1];
    const int64_t e0 = s0 + (int64_t)(chunk - chunk_offsets[s]) * CQ_CHUNK;
    const int64_t e1 = min(e0 + (int64_t)CQ_CHUNK, s1);
    const float* xr = x + z * x_cs;
    const float* br = base ? base + z * b_cs : nullptr;
    float* orow = out ? out + z * o_cs : nullptr;
    uint8_t* krow = keep ? keep + z * k_cs : nullptr;
    __shared__ uint32_t wcnt[4];
    __shared__ uint32_t s_before;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t before = 0;  // equal keys at lower indices of this segment (ranked mode)
    if (ranked) {
        if (threadIdx.x == 0) {
            uint32_t c = 0;
            for (int q = chunk_offsets[s]; q < chunk; ++q)
                c += chunk_hist[((int64_t)z * nchunks + q) * 256 + (T & 255u)];
            s_before = c;
        }
        __syncthreads();
        before = s_before;
    }
    for (int64_t t0 = e0; t0 < e1; t0 += 256) {
        const int64_t i = t0 + threadIdx.x;
        const bool in = i < e1;
        const float v = in ? delta_at(xr, br, i) : 0.f;
        const uint32_t key = mag_key(v);
        const bool eq = in && key == T;
        bool k = in && key > T;
        if (ranked) {
            const uint64_t m = __ballot(eq);
            const uint32_t lower = __popcll(m & ((1ull << lane) - 1ull));
            __syncthreads();
            if (lane == 0) wcnt[wid] = __popcll(m);
            __syncthreads();
            uint32_t off = before;
            for (int w = 0; w < wid; ++w) off += wcnt[w];
            k = k || (eq && off + lower < st.kr);
            before += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        } else {
            k = k || eq;
        }
        if (in) {
            if (krow) krow[i] = (uint8_t)k;
            if (orow) {
                const float d = k ? v : 0.f;
                orow[i] = br ? br[i] + d : d;
            }
        }
    }
}

}  // namespace fh

using namespace fh;

extern "C" int64_t fh_compress_chunk_elems(void) { return CQ_CHUNK; }

extern "C" int64_t fh_quantize_workspace(int32_t nclients, int32_t nchunks) {
    return (int64_t)nclients * nchunks * (int64_t)sizeof(float2);
}

extern "C" int fh_quantize_rows(const float* x, int64_t x_cs, const float* base, int64_t base_cs,
                                float* out, int64_t out_cs, uint8_t* codes, int64_t codes_cs,
                                int32_t nclients, const int64_t* seg_offsets,
                                const int32_t* chunk_offsets, int32_t nseg, int32_t nchunks,
                                int32_t bits, int32_t symmetric, double* scale_out,
                                int64_t* zp_out, void* ws, size_t ws_bytes, void* stream) {
    FH_REQUIRE(nclients >= 0 && nseg > 0 && nchunks >= nseg, "quantize_rows: bad shape");
    FH_REQUIRE(bits >= 1 && bits <= 16, "quantize_rows: bits must be in [1, 16] (got %d)", bits);
    FH_REQUIRE(!codes || bits <= 8, "quantize_rows: uint8 codes need bits <= 8");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && seg_offsets && chunk_offsets, "quantize_rows: null pointer");
    FH_REQUIRE(ws && (int64_t)ws_bytes >= fh_quantize_workspace(nclients, nchunks),
               "quantize_rows: workspace too small");
    float2* partial = reinterpret_cast<float2*>(ws);
    hipStream_t st = as_stream(stream);
    dim3 grid(nchunks, nclients);
    FH_LAUNCH(quant_minmax_kernel, grid, dim3(256), 0, st, x, x_cs, base, base_cs,
                       seg_offsets, chunk_offsets, nseg, nchunks, partial);
    FH_LAUNCH_CHECK("quantize_rows/minmax");
    FH_LAUNCH(quant_apply_kernel, grid, dim3(256), 0, st, x, x_cs, base, base_cs, out,
                       out_cs, codes, codes_cs, seg_offsets, chunk_offsets, nseg, nchunks,
                       partial, 1 << bits, symmetric, scale_out, zp_out);
    FH_LAUNCH_CHECK("quantize_rows/apply");
    return FH_OK;
}

extern "C" int64_t fh_topk_workspace(int32_t nclients, int32_t nseg, int32_t nchunks) {
    return (int64_t)nclients * ((int64_t)nseg * (256 * sizeof(uint32_t) + sizeof(TopkState)) +
                                (int64_t)nchunks * 256 * sizeof(uint32_t));
}

extern "C" int fh_topk_rows(const float* x, int64_t x_cs, const float* base, int64_t base_cs,
                            float* out, int64_t out_cs, uint8_t* keep, int64_t keep_cs,
                            int32_t nclients, const int64_t* seg_offsets,
                            const int32_t* chunk_offsets, const int64_t* seg_k, int32_t nseg,
                            int32_t nchunks, void* ws, size_t ws_bytes, void* stream) {
    FH_REQUIRE(nclients >= 0 && nseg > 0 && nchunks >= nseg, "topk_rows: bad shape");
    if (nclients == 0) return FH_OK;
    FH_REQUIRE(x && seg_offsets && chunk_offsets && seg_k, "topk_rows: null pointer");
    FH_REQUIRE(ws && (int64_t)ws_bytes >= fh_topk_workspace(nclients, nseg, nchunks),
               "topk_rows: workspace too small");
    uint32_t* hist = reinterpret_cast<uint32_t*>(ws);
    TopkState* state = reinterpret_cast<TopkState*>(hist + (int64_t)nclients * nseg * 256);
    uint32_t* chunk_hist = reinterpret_cast<uint32_t*>(state + (int64_t)nclients * nseg);
    hipStream_t st = as_stream(stream);
    if (hipMemsetAsync(hist, 0, (size_t)nclients * nseg * 256 * sizeof(uint32_t), st) != hipSuccess) {
        set_error("topk_rows: memset failed");
        return FH_E_LAUNCH;
    }
    dim3 grid(nchunks, nclients), sgrid(nseg, nclients);
    for (int r = 0; r < 4; ++r) {
        FH_LAUNCH(topk_hist_kernel, grid, dim3(256), 0, st, x, x_cs, base, base_cs,
                           seg_offsets, chunk_offsets, nseg, state, hist, r,
                           r == 3 ? chunk_hist : nullptr, nchunks);
        FH_LAUNCH_CHECK("topk_rows/hist");
        FH_LAUNCH(topk_select_kernel, sgrid, dim3(64), 0, st, seg_k, nseg, state, hist,
                           r);
        FH_LAUNCH_CHECK("topk_rows/select");
    }
    FH_LAUNCH(topk_apply_kernel, grid, dim3(256), 0, st, x, x_cs, base, base_cs, out,
                       out_cs, keep, keep_cs, seg_offsets, chunk_offsets, nseg, state,
                       chunk_hist, nchunks);
    FH_LAUNCH_CHECK("topk_rows/apply");
    return FH_OK;
}
