// splitbn.h — a split direct convolution's reduction left to the BatchNorm call that follows it
// (r06, fh_conv_bn_defer).
//
// A split FWD / DGRAD launch with a statistics epilogue (conv.hip run_dconv) normally leaves a
// [client][split][M][Nfull] slab that splitk_epilogue_kernel sums — writing the output and one
// fp64 statistics pair per (client, channel, 256-element tile) — after which the BatchNorm call
// (finalize / max-pool finalize / backward apply) merges the tiles per channel.  Both passes
// are channel-local, so with the defer armed the conv records its epilogue here instead and the
// BatchNorm call runs both as ONE launch of one 1024-thread workgroup per (channel, client)
// (bn.hip split_bnfin_kernel / split_bnbwd_kernel): the slab summed in split order, the tiles
// formed exactly as the epilogue forms them and merged exactly as the BN kernels merge them —
// every stored value bit-identical to the two-launch path.  Anything else that finds the record
// pending launches the skipped epilogue first (sbn_materialize).
#pragma once

#include "fh_common.h"

namespace fh {

// one client-channel's elements the fused launch keeps in LDS (batch x plane pixels)
constexpr int kSbnMaxElems = 8192;
constexpr int kSbnMaxTiles = kSbnMaxElems / 256;

struct SplitBnRec {
    bool pending = false;
    int op = 0;  // 0 FWD (statistics of y), 1 DGRAD (BN-backward statistics of the masked dX)
    const float* part = nullptr;  // the slab
    int splits = 0, M = 0, sp = 0, batch = 0, nclients = 0;
    int64_t Nfull = 0;
    float* out = nullptr;  // the epilogue's output (y, or the pooled / masked gradient)
    int64_t out_cs = 0;
    const float* bias = nullptr;  // FWD
    int64_t b_cs = 0;
    const int32_t* counts = nullptr;
    double* bn_part = nullptr;  // the statistics tiles the epilogue would write (the key)
    int bn_tiles = 0;
    // DGRAD: the BN in front of the conv (relu(bnx * scale + shift)), routed through a 2x2
    // max-pool (+ dropout keep-mask) when pidx is non-null (pw: pooled map width)
    const float* bnx = nullptr;
    int64_t bnx_cs = 0;
    const float* bn_scale = nullptr;
    const float* bn_shift = nullptr;
    int64_t bns_cs = 0;
    const float* bn_mean = nullptr;
    const uint8_t* pidx = nullptr;
    const uint8_t* pmask = nullptr;
    int64_t pi_cs = 0, pm_cs = 0;
    float pscale = 1.f;
    int pw = 0;
    hipStream_t st = nullptr;
};

// conv.hip: the calling thread's record (pending or not) and the skipped epilogue launch
SplitBnRec& sbn_rec();
int sbn_materialize();
// bn.hip: fused launches issued on this thread (fh_conv_bn_defer_status)
int64_t sbn_taken();

}  // namespace fh
