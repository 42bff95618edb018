// program.hip — step programs: a training step recorded once as a flat list of kernel
// launches and re-issued with hipLaunchKernel on the lane's own stream.
//
// Why.  Concurrent client lanes (fedhip/lanes.py) each issue one step per global step on
// their own stream.  Re-issuing the step's kernels with hipLaunchKernel instead of
// hipGraphLaunch, with the per-step input row moved by a kernel instead of a device-to-
// device hipMemcpyAsync, measured +1.3 % client-images/s on KT (3 lanes,
// profiles/r01_v10/launch_modes.txt) at ~2-3 us of host time per kernel, which the host
// hides (it runs tens of steps ahead).
//
// Ownership.  The program is recorded by the library's own launch path (FH_LAUNCH in
// fh_common.h): while a recorder is active on the calling thread every kernel launch
// appends {kernel, grid, block, LDS bytes, a private typed copy of its arguments}.  Nothing
// is borrowed from a HIP graph node or from runtime storage, so the program stays valid
// for exactly as long as the device buffers its arguments point at (the caller keeps
// those alive — fedhip/engine.py holds them with the program).  The host side records
// while the same step is captured into a HIP graph and compares the two: a step that
// contains anything the recorder cannot see (a memset, a copy, a kernel launched outside
// libfedhip) makes the recording invalid and the caller replays the graph instead.
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "fh_common.h"

namespace fh {

struct RecordedKernel {
    const void* func;
    dim3 grid, block;
    size_t shmem;
    std::unique_ptr<KernelArgs> args;
};

// r06: argument words of the recorded launches that point into the step's per-step input
// slot (fh_program_relocate); fh_program_launch_at rewrites them to another row first.
struct Reloc {
    uint64_t* word;
    uint64_t off;
};

struct Recorder {
    std::vector<RecordedKernel> kernels;
    std::vector<Reloc> relocs;
    Recorder* prev = nullptr;  // recorders nest per thread (never in practice)
};

thread_local Recorder* g_recorder = nullptr;

void record_kernel(Recorder* r, const void* func, dim3 grid, dim3 block, size_t shmem,
                   KernelArgs* args) {
    r->kernels.push_back(RecordedKernel{func, grid, block, shmem,
                                        std::unique_ptr<KernelArgs>(args)});
}

}  // namespace fh

using fh::Recorder;

#define FH_HIPCHK(expr, what)                                                  \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            fh::set_error("%s: %s", what, hipGetErrorString(e_));              \
            return FH_E_LAUNCH;                                                \
        }                                                                      \
    } while (0)

extern "C" int fh_record_begin(void** program_out) {
    if (!program_out) {
        fh::set_error("fh_record_begin: null argument");
        return FH_E_INVALID;
    }
    auto* r = new Recorder();
    r->prev = fh::g_recorder;
    fh::g_recorder = r;
    *program_out = r;
    return FH_OK;
}

extern "C" int fh_record_end(void* program, int32_t* kernels_out) {
    auto* r = (Recorder*)program;
    if (!r || fh::g_recorder != r) {
        fh::set_error("fh_record_end: not the active recorder of this thread");
        return FH_E_INVALID;
    }
    fh::g_recorder = r->prev;
    r->prev = nullptr;
    if (kernels_out) *kernels_out = (int32_t)r->kernels.size();
    return FH_OK;
}

// Kernel / other node counts of a captured graph (the host compares them with a
// recording of the same step: equal kernel counts and no other work node = complete).
extern "C" int fh_graph_node_counts(void* graph, int32_t* kernels_out, int32_t* others_out) {
    if (!graph || !kernels_out || !others_out) {
        fh::set_error("fh_graph_node_counts: null argument");
        return FH_E_INVALID;
    }
    hipGraph_t g = (hipGraph_t)graph;
    size_t n = 0;
    FH_HIPCHK(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    if (n) FH_HIPCHK(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
    int32_t k = 0, o = 0;
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        FH_HIPCHK(hipGraphNodeGetType(nodes[i], &t), "hipGraphNodeGetType");
        if (t == hipGraphNodeTypeKernel) ++k;
        else if (t != hipGraphNodeTypeEmpty) ++o;
    }
    *kernels_out = k;
    *others_out = o;
    return FH_OK;
}

// The recording is a faithful copy of the captured graph: the graph holds no work node
// other than kernels (no memset / copy / foreign node types) and its kernels are the
// recorded ones — the same function for every launch, compared as multisets of kernel
// functions (node order in a graph is not launch order).  A libfedhip launch recorded on a
// stream that was not being captured, or a foreign kernel captured beside the library's,
// fails the comparison even when the counts agree.
extern "C" int fh_program_matches_graph(void* program, void* graph, int32_t* match_out) {
    auto* r = (Recorder*)program;
    if (!r || !graph || !match_out) {
        fh::set_error("fh_program_matches_graph: null argument");
        return FH_E_INVALID;
    }
    *match_out = 0;
    hipGraph_t g = (hipGraph_t)graph;
    size_t n = 0;
    FH_HIPCHK(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    if (n) FH_HIPCHK(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
    std::vector<const void*> got, want;
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        FH_HIPCHK(hipGraphNodeGetType(nodes[i], &t), "hipGraphNodeGetType");
        if (t == hipGraphNodeTypeEmpty) continue;
        if (t != hipGraphNodeTypeKernel) return FH_OK;  // a memset / copy / other node
        hipKernelNodeParams kp{};
        FH_HIPCHK(hipGraphKernelNodeGetParams(nodes[i], &kp), "hipGraphKernelNodeGetParams");
        got.push_back(kp.func);
    }
    for (const auto& k : r->kernels) want.push_back(k.func);
    std::sort(got.begin(), got.end());
    std::sort(want.begin(), want.end());
    *match_out = got == want ? 1 : 0;
    return FH_OK;
}

extern "C" int fh_program_launch(void* program, void* stream) {
    auto* r = (Recorder*)program;
    if (!r) {
        fh::set_error("fh_program_launch: null program");
        return FH_E_INVALID;
    }
    if (fh::g_recorder == r) {
        fh::set_error("fh_program_launch: program is still recording");
        return FH_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    for (const auto& k : r->kernels)
        FH_HIPCHK(hipLaunchKernel(k.func, k.grid, k.block, k.args->params, k.shmem, st),
                  "fh_program_launch");
    return FH_OK;
}

// r06: relocation of the per-step input slot.  A step program's kernels read the step's
// inputs (batch indices, counts, reset flags, Philox key block, Adam scalars) from one fixed
// slot that a copy_bytes launch refills from the round's row g before every step — one more
// ~4.5 us dependent launch per step on every lane.  fh_program_relocate finds every 8-byte
// argument word (struct fields included) equal to one of the slot's view pointers `ptrs`; any
// other word pointing into [base, base + len) fails the relocation (found = -1: the caller
// keeps copying).  fh_program_launch_at rewrites those words to the same offsets in another
// row (hipLaunchKernel copies the argument bytes at enqueue) and issues the program: the
// kernels read row g itself and the copy launch disappears.
extern "C" int fh_program_relocate(void* program, const uint64_t* ptrs, int32_t nptrs,
                                   uint64_t base, int64_t len, int32_t* found) {
    auto* r = (Recorder*)program;
    if (!r || !found || (nptrs > 0 && !ptrs) || nptrs < 0 || len <= 0 || fh::g_recorder == r) {
        fh::set_error("fh_program_relocate: bad arguments");
        return FH_E_INVALID;
    }
    for (int j = 0; j < nptrs; ++j)
        if (ptrs[j] < base || ptrs[j] >= base + (uint64_t)len) {
            fh::set_error("fh_program_relocate: pointer %d outside the slot", j);
            return FH_E_INVALID;
        }
    r->relocs.clear();
    for (auto& k : r->kernels) {
        const fh::KernelArgs* a = k.args.get();
        for (int i = 0; i < a->nargs; ++i) {
            char* p = (char*)a->params[i];
            for (size_t o = 0; o + 8 <= a->sizes[i]; o += 8) {
                if (((uintptr_t)(p + o)) % 8) continue;
                uint64_t v;
                memcpy(&v, p + o, 8);
                if (v < base || v >= base + (uint64_t)len) continue;
                bool known = false;
                for (int j = 0; j < nptrs && !known; ++j) known = v == ptrs[j];
                if (!known) {  // a pointer into the slot the caller did not declare
                    r->relocs.clear();
                    *found = -1;
                    return FH_OK;
                }
                r->relocs.push_back(fh::Reloc{(uint64_t*)(p + o), v - base});
            }
        }
    }
    *found = (int32_t)r->relocs.size();
    return FH_OK;
}

extern "C" int fh_program_launch_at(void* program, void* stream, uint64_t base) {
    auto* r = (Recorder*)program;
    if (!r || fh::g_recorder == r || r->relocs.empty() || !base) {
        fh::set_error("fh_program_launch_at: no relocatable program");
        return FH_E_INVALID;
    }
    for (const auto& rl : r->relocs) *rl.word = base + rl.off;
    return fh_program_launch(program, stream);
}

// Per-step input row -> the fixed slot the step kernels read (a kernel: part of the
// measured program-mode gain over hipMemcpyAsync device-to-device).
__global__ void __launch_bounds__(256) copy_bytes_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, int64_t n16) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
        dst[i] = src[i];
}

extern "C" int fh_copy_bytes(const void* src, void* dst, int64_t nbytes, void* stream) {
    if (nbytes < 0 || nbytes % 16 || (uintptr_t)src % 16 || (uintptr_t)dst % 16) {
        fh::set_error("fh_copy_bytes: need 16-B aligned pointers and size (got %lld)",
                      (long long)nbytes);
        return FH_E_INVALID;
    }
    if (!nbytes) return FH_OK;
    const int64_t n16 = nbytes / 16;
    const int blocks = (int)std::min<int64_t>((n16 + 255) / 256, 1024);
    FH_LAUNCH(copy_bytes_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
              (const uint4*)src, (uint4*)dst, n16);
    return FH_OK;
}

extern "C" int fh_program_destroy(void* program) {
    auto* r = (Recorder*)program;
    if (r && fh::g_recorder == r) {
        fh::set_error("fh_program_destroy: program is still recording");
        return FH_E_INVALID;
    }
    delete r;
    return FH_OK;
}
