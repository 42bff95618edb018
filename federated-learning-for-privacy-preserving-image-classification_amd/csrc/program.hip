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
//
// Launch-group timing (r05).  bench.py's roofline is the average duration of one launch
// shape over the TIMED rounds, measured with HIP events on the launch stream.  A launch
// shape is one fedhip.ops call (its kernel, plus a split-K reduction when it has one), so
// the host brackets every such call with fh_tag_begin(tag) / fh_tag_end(): a recording marks
// the call's first and last kernel with the tag, and a replay of the program — or an eager
// launch — records a start event before the group's first kernel and an end event after its
// last when that tag is enabled (fh_timing_enable).  Nothing is recorded for tags that are
// not enabled, and with timing off a replay issues exactly the recorded kernels.
#include <algorithm>
#include <memory>
#include <mutex>
#include <unordered_set>
#include <vector>

#include "fh_common.h"

namespace fh {

struct RecordedKernel {
    const void* func;
    dim3 grid, block;
    size_t shmem;
    std::unique_ptr<KernelArgs> args;
    int tag = 0;               // launch group (fh_tag_begin) this kernel belongs to, 0 none
    bool gbeg = false, gend = false;  // first / last kernel of its group
};

struct Recorder {
    std::vector<RecordedKernel> kernels;
    Recorder* prev = nullptr;  // recorders nest per thread (never in practice)
};

thread_local Recorder* g_recorder = nullptr;

// ---- launch-group tags and timing
thread_local int g_tag = 0;           // the current group's tag (0: none)
thread_local size_t g_tag_first = 0;  // recorder index of the group's first kernel
thread_local int g_tag_timed = 0;     // g_tag is enabled: eager launches are timed
thread_local hipEvent_t g_tag_ev0 = nullptr, g_tag_ev1 = nullptr;  // eager group's events
thread_local hipStream_t g_tag_last = nullptr;  // stream of the eager group's last launch

struct TimedLaunch {
    int tag;
    hipEvent_t a, b;
};
struct Timing {
    std::mutex mu;
    bool on = false;
    std::unordered_set<int> tags;
    std::vector<hipEvent_t> pool;  // created by fh_timing_enable, reused after a reset
    size_t next = 0;
    int64_t dropped = 0;           // groups not timed: the pool ran out
    std::vector<TimedLaunch> recs;
    bool enabled(int tag) {
        std::lock_guard<std::mutex> g(mu);
        return on && tags.count(tag) != 0;
    }
    bool take(hipEvent_t& a, hipEvent_t& b) {
        std::lock_guard<std::mutex> g(mu);
        if (next + 2 > pool.size()) {
            ++dropped;
            return false;
        }
        a = pool[next++];
        b = pool[next++];
        return true;
    }
    void add(int tag, hipEvent_t a, hipEvent_t b) {
        std::lock_guard<std::mutex> g(mu);
        recs.push_back(TimedLaunch{tag, a, b});
    }
};
Timing& timing() {
    static Timing* t = new Timing();  // never destroyed: events outlive interpreter teardown
    return *t;
}

void record_kernel(Recorder* r, const void* func, dim3 grid, dim3 block, size_t shmem,
                   KernelArgs* args) {
    RecordedKernel k{func, grid, block, shmem, std::unique_ptr<KernelArgs>(args)};
    if (g_tag) {
        k.tag = g_tag;
        k.gbeg = r->kernels.size() == g_tag_first;
    }
    r->kernels.push_back(std::move(k));
}

// an eager launch inside a timed group: the start event ahead of the group's first kernel
void tag_before_launch(hipStream_t st) {
    if (!g_tag_ev0) {
        hipEvent_t a, b;
        if (!timing().take(a, b)) {
            g_tag_timed = 0;
            return;
        }
        (void)hipEventRecord(a, st);
        g_tag_ev0 = a;
        g_tag_ev1 = b;
    }
    g_tag_last = st;
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
    fh::Timing& tm = fh::timing();
    bool timed_any;
    {
        std::lock_guard<std::mutex> g(tm.mu);
        timed_any = tm.on && !tm.tags.empty();
    }
    if (!timed_any) {
        for (const auto& k : r->kernels)
            FH_HIPCHK(hipLaunchKernel(k.func, k.grid, k.block, k.args->params, k.shmem, st),
                      "fh_program_launch");
        return FH_OK;
    }
    hipEvent_t ea = nullptr, eb = nullptr;
    int etag = 0;
    for (const auto& k : r->kernels) {
        if (k.gbeg && tm.enabled(k.tag) && tm.take(ea, eb)) {
            FH_HIPCHK(hipEventRecord(ea, st), "fh_program_launch event");
            etag = k.tag;
        }
        FH_HIPCHK(hipLaunchKernel(k.func, k.grid, k.block, k.args->params, k.shmem, st),
                  "fh_program_launch");
        if (k.gend && etag == k.tag && ea) {
            FH_HIPCHK(hipEventRecord(eb, st), "fh_program_launch event");
            tm.add(etag, ea, eb);
            ea = eb = nullptr;
            etag = 0;
        }
    }
    return FH_OK;
}

// ---- launch-group tags (see the header comment) -----------------------------------------
extern "C" int fh_tag_begin(int32_t tag) {
    if (tag <= 0) {
        fh::set_error("fh_tag_begin: tag %d (must be > 0)", tag);
        return FH_E_INVALID;
    }
    fh::g_tag = tag;
    fh::g_tag_first = fh::g_recorder ? fh::g_recorder->kernels.size() : 0;
    fh::g_tag_timed = !fh::g_recorder && fh::timing().enabled(tag) ? 1 : 0;
    fh::g_tag_ev0 = fh::g_tag_ev1 = nullptr;
    fh::g_tag_last = nullptr;
    return FH_OK;
}

// retag the open group (a DGRAD call that issued the held WGRAD with it: the dual launch)
extern "C" int fh_tag_retag(int32_t tag) {
    if (tag <= 0 || !fh::g_tag) {
        fh::set_error("fh_tag_retag: tag %d, open group %d", tag, fh::g_tag);
        return FH_E_INVALID;
    }
    if (fh::g_recorder)
        for (size_t i = fh::g_tag_first; i < fh::g_recorder->kernels.size(); ++i)
            fh::g_recorder->kernels[i].tag = tag;
    fh::g_tag = tag;
    return FH_OK;
}

extern "C" int fh_tag_end(void) {
    if (fh::g_recorder && fh::g_tag) {
        auto& ks = fh::g_recorder->kernels;
        if (ks.size() > fh::g_tag_first) ks.back().gend = true;
    }
    if (fh::g_tag_ev0 && fh::g_tag_last) {  // an eager timed group
        FH_HIPCHK(hipEventRecord(fh::g_tag_ev1, fh::g_tag_last), "fh_tag_end event");
        fh::timing().add(fh::g_tag, fh::g_tag_ev0, fh::g_tag_ev1);
    }
    fh::g_tag = 0;
    fh::g_tag_timed = 0;
    fh::g_tag_ev0 = fh::g_tag_ev1 = nullptr;
    fh::g_tag_last = nullptr;
    return FH_OK;
}

// timing on for the given tags (n = 0: off), with `reserve` event pairs; drops every
// earlier record
extern "C" int fh_timing_enable(const int32_t* tags, int32_t n, int32_t reserve) {
    if (n < 0 || reserve < 0 || (n && !tags)) {
        fh::set_error("fh_timing_enable: bad arguments");
        return FH_E_INVALID;
    }
    fh::Timing& tm = fh::timing();
    std::lock_guard<std::mutex> g(tm.mu);
    tm.tags.clear();
    for (int i = 0; i < n; ++i) tm.tags.insert(tags[i]);
    while (tm.pool.size() < (size_t)2 * reserve) {
        hipEvent_t e;
        FH_HIPCHK(hipEventCreate(&e), "hipEventCreate");
        tm.pool.push_back(e);
    }
    tm.next = 0;
    tm.dropped = 0;
    tm.recs.clear();
    tm.on = n > 0;
    return FH_OK;
}

// launches timed for `tag` since fh_timing_enable, their summed duration (waits for the
// events) and the groups not timed for want of events
extern "C" int fh_timing_collect(int32_t tag, int64_t* launches, double* total_ms,
                                 int64_t* dropped) {
    if (!launches || !total_ms || !dropped) {
        fh::set_error("fh_timing_collect: null pointer");
        return FH_E_INVALID;
    }
    fh::Timing& tm = fh::timing();
    std::lock_guard<std::mutex> g(tm.mu);
    int64_t n = 0;
    double ms = 0.0;
    for (const auto& r : tm.recs) {
        if (r.tag != tag) continue;
        FH_HIPCHK(hipEventSynchronize(r.b), "hipEventSynchronize");
        float t = 0.f;
        FH_HIPCHK(hipEventElapsedTime(&t, r.a, r.b), "hipEventElapsedTime");
        ++n;
        ms += t;
    }
    *launches = n;
    *total_ms = ms;
    *dropped = tm.dropped;
    return FH_OK;
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
