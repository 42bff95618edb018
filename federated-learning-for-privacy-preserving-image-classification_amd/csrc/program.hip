// program.hip — step programs: a captured training step replayed as plain kernel
// launches on the lane's own stream.
//
// Why.  Concurrent client lanes (fedhip/lanes.py) each replay one captured step per
// global step on their own stream.  Replaying the kernel list with hipLaunchKernel
// instead of hipGraphLaunch, with the per-step input row moved by a kernel instead of a
// device-to-device hipMemcpyAsync, measured +1.3 % client-images/s on KT (3 lanes,
// profiles/r01_v10/launch_modes.txt) at ~2-3 us of host time per kernel, which the host
// hides (it runs tens of steps ahead).  The kernels, arguments and order are the graph's,
// so results are identical by construction.  (Under rocprofv3 --kernel-trace, lanes
// replaying graphs or programs appear to advance in lockstep; HIP-event timelines
// without the profiler show them overlapping — trust the events.)
#include <vector>

#include "fh_common.h"

namespace fh {

struct ProgOp {
    int kind;  // 0 kernel, 1 memset, 2 memcpy
    hipKernelNodeParams k;
    hipMemsetParams ms;
    hipMemcpy3DParms mc;
};

struct Program {
    std::vector<ProgOp> ops;
    int kernels = 0;
};

}  // namespace fh

using fh::ProgOp;
using fh::Program;

#define FH_HIPCHK(expr, what)                                                  \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess) {                                                \
            fh::set_error("%s: %s", what, hipGetErrorString(e_));              \
            return FH_E_LAUNCH;                                                \
        }                                                                      \
    } while (0)

extern "C" int fh_program_from_graph(void* graph, void** program_out, int32_t* kernels_out) {
    if (!graph || !program_out) {
        fh::set_error("fh_program_from_graph: null argument");
        return FH_E_INVALID;
    }
    hipGraph_t g = (hipGraph_t)graph;
    size_t n = 0;
    FH_HIPCHK(hipGraphGetNodes(g, nullptr, &n), "hipGraphGetNodes");
    std::vector<hipGraphNode_t> nodes(n);
    if (n) FH_HIPCHK(hipGraphGetNodes(g, nodes.data(), &n), "hipGraphGetNodes");
    size_t ne = 0;
    FH_HIPCHK(hipGraphGetEdges(g, nullptr, nullptr, &ne), "hipGraphGetEdges");
    std::vector<hipGraphNode_t> from(ne), to(ne);
    if (ne) FH_HIPCHK(hipGraphGetEdges(g, from.data(), to.data(), &ne), "hipGraphGetEdges");
    // Kahn's order (ties by capture order): one serial stream honours every edge
    auto idx = [&](hipGraphNode_t x) {
        for (size_t i = 0; i < n; ++i)
            if (nodes[i] == x) return (int)i;
        return -1;
    };
    std::vector<int> indeg(n, 0);
    std::vector<std::vector<int>> succ(n);
    for (size_t e = 0; e < ne; ++e) {
        const int a = idx(from[e]), b = idx(to[e]);
        if (a < 0 || b < 0) {
            fh::set_error("fh_program_from_graph: edge to an unknown node");
            return FH_E_INVALID;
        }
        succ[a].push_back(b);
        ++indeg[b];
    }
    std::vector<int> order, ready;
    for (size_t i = 0; i < n; ++i)
        if (!indeg[i]) ready.push_back((int)i);
    while (!ready.empty()) {
        auto it = std::min_element(ready.begin(), ready.end());
        const int v = *it;
        ready.erase(it);
        order.push_back(v);
        for (int s : succ[v])
            if (--indeg[s] == 0) ready.push_back(s);
    }
    if (order.size() != n) {
        fh::set_error("fh_program_from_graph: graph has a cycle");
        return FH_E_INVALID;
    }
    auto* prog = new Program();
    for (int v : order) {
        hipGraphNodeType t;
        hipError_t e = hipGraphNodeGetType(nodes[v], &t);
        ProgOp op{};
        if (e == hipSuccess && t == hipGraphNodeTypeKernel) {
            e = hipGraphKernelNodeGetParams(nodes[v], &op.k);
            if (e == hipSuccess && (!op.k.kernelParams || op.k.extra)) {
                delete prog;
                fh::set_error("fh_program_from_graph: kernel node without kernelParams");
                return FH_E_UNSUPPORTED;
            }
            op.kind = 0;
            ++prog->kernels;
        } else if (e == hipSuccess && t == hipGraphNodeTypeMemset) {
            e = hipGraphMemsetNodeGetParams(nodes[v], &op.ms);
            op.kind = 1;
        } else if (e == hipSuccess && t == hipGraphNodeTypeMemcpy) {
            e = hipGraphMemcpyNodeGetParams(nodes[v], &op.mc);
            op.kind = 2;
        } else if (e == hipSuccess && t == hipGraphNodeTypeEmpty) {
            continue;
        } else if (e == hipSuccess) {
            delete prog;
            fh::set_error("fh_program_from_graph: unsupported node type %d", (int)t);
            return FH_E_UNSUPPORTED;
        }
        if (e != hipSuccess) {
            delete prog;
            fh::set_error("fh_program_from_graph: %s", hipGetErrorString(e));
            return FH_E_LAUNCH;
        }
        prog->ops.push_back(op);
    }
    *program_out = prog;
    if (kernels_out) *kernels_out = prog->kernels;
    return FH_OK;
}

extern "C" int fh_program_launch(void* program, void* stream) {
    auto* prog = (Program*)program;
    if (!prog) {
        fh::set_error("fh_program_launch: null program");
        return FH_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    for (const ProgOp& op : prog->ops) {
        if (op.kind == 0) {
            FH_HIPCHK(hipLaunchKernel(op.k.func, op.k.gridDim, op.k.blockDim, op.k.kernelParams,
                                      op.k.sharedMemBytes, st),
                      "fh_program_launch kernel");
        } else if (op.kind == 1) {
            const hipMemsetParams& m = op.ms;
            if (m.elementSize == 4 && m.height <= 1) {
                FH_HIPCHK(hipMemsetD32Async((hipDeviceptr_t)m.dst, m.value, m.width, st),
                          "fh_program_launch memset");
            } else if (m.elementSize == 1) {
                FH_HIPCHK(hipMemset2DAsync(m.dst, m.pitch ? m.pitch : m.width, (int)m.value,
                                           m.width, m.height ? m.height : 1, st),
                          "fh_program_launch memset");
            } else {
                fh::set_error("fh_program_launch: memset element size %u", m.elementSize);
                return FH_E_UNSUPPORTED;
            }
        } else {
            FH_HIPCHK(hipMemcpy3DAsync(&op.mc, st), "fh_program_launch memcpy");
        }
    }
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
    hipLaunchKernelGGL(copy_bytes_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, (uint4*)dst, n16);
    FH_HIPCHK(hipGetLastError(), "fh_copy_bytes");
    return FH_OK;
}

extern "C" int fh_program_destroy(void* program) {
    delete (Program*)program;
    return FH_OK;
}
