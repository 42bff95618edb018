/*
 * fedhip.h — C ABI of libfedhip.so, the MI355X (gfx950) hot path for
 * per-client CNN training, update-level differential privacy and FedAvg.
 *
 * Every entry point:
 *   - returns FH_OK (0) or a negative FH_E_* code; fh_last_error() gives a
 *     thread-local message for the last failure on the calling thread;
 *   - takes caller-owned DEVICE pointers (fp32 unless stated), contiguous,
 *     with element strides spelled out; no hidden allocation, no host sync;
 *   - launches on `stream` (a hipStream_t passed as void*; NULL = default).
 *
 * "Packed" tensors hold many simulated clients: client slot z of a tensor
 * `t` with client stride `t_cs` starts at t + z * t_cs.  Clients are packed
 * into slots sorted by descending step count, so the clients still active at
 * a given step are always the prefix [0, nclients).  `counts[z]` (device
 * int32, may be NULL = all `batch` valid) is the number of valid images of
 * client z in this step — the reference's partial last batch
 * (DataLoader drop_last=False, src/shared/training.py:184).
 *
 * Reference interfaces replaced (file:line in the reference repository):
 *   fh_fedavg_weighted_sum   src/aggregation/fedavg.py:267-289 (_weighted_average)
 *   fh_update_stats          src/shared/validation.py:72-91   (_validate_model_weights)
 *   fh_dp_delta_sqnorm       src/shared/privacy.py:119-123    (GradientClipper norm)
 *                            + src/client/federated_trainer.py:438-443 (delta)
 *   fh_dp_clip_coef          src/shared/privacy.py:123-140, 209 (clip decision, sigma)
 *   fh_dp_apply              src/shared/privacy.py:127-133, 212, 244-245
 *                            + src/client/federated_trainer.py:454-459
 *   fh_sgd_step / fh_adam_step   src/shared/training.py:244-255 + torch.optim
 *   fh_conv2d_* / fh_linear_*    nn.Conv2d / nn.Linear in src/shared/models_pytorch.py
 *   fh_bn_*                  nn.BatchNorm2d (models_pytorch.py:108-120, 176-187)
 *   fh_maxpool2_*            nn.MaxPool2d(2,2) (models_pytorch.py:72,123)
 *   fh_dropout_*             nn.Dropout (models_pytorch.py:75,124)
 *   fh_ce_fwd_bwd            nn.CrossEntropyLoss + metrics (training.py:90,193,200-203)
 *   fh_eval_metrics          LocalTrainer.evaluate_model metrics (training.py:307-360)
 *   fh_quantize_rows         QuantizationCompressor (compression.py:123-247)
 *   fh_topk_rows             TopKSparsificationCompressor (compression.py:250-368)
 */
#ifndef FEDHIP_H_
#define FEDHIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FH_OK 0
#define FH_E_INVALID (-1)     /* bad argument / shape */
#define FH_E_LAUNCH (-2)      /* HIP launch or runtime failure */
#define FH_E_UNSUPPORTED (-3) /* shape/config outside what the kernels cover */

const char* fh_last_error(void);
int fh_version(void);

/* ---------------- FedAvg (fedavg.py:267-289) ------------------------------
 * out[j] = (accumulate ? out[j] : 0) + sum_{k=0..C-1} fl32(w[k]) * rows[idx[k]*row_stride + j]
 * evaluated sequentially in k with a rounded multiply followed by a rounded
 * add (never a fused multiply-add): bit-exact with the reference's
 * `aggregated[l] += weight * layer` loop over the client list.
 * row_index (device int32[C]) may be NULL (identity); weights: device float[C]. */
int fh_fedavg_weighted_sum(const float* rows, int64_t row_stride, const int32_t* row_index,
                           const float* weights, int32_t num_clients, int64_t P, float* out,
                           int32_t accumulate, void* stream);

/* Per client, per parameter tensor (segment [seg_off[t], seg_off[t+1]) of a row):
 * max |w| and a non-finite flag (validation.py:81-91). seg_offsets: device int64[nseg+1]. */
int fh_update_stats(const float* rows, int64_t row_stride, int32_t num_clients,
                    const int64_t* seg_offsets, int32_t nseg, float* seg_absmax,
                    int32_t* seg_nonfinite, void* stream);

/* ---------------- update-level DP (privacy.py:107-144, 183-254) ----------
 * delta = fl32(local - global) (global may be NULL: delta = local).
 * seg_sqnorm[z*nseg+t] = sum over segment t of delta^2, accumulated in fp64. */
int fh_dp_delta_sqnorm(const float* local, int64_t local_stride, const float* global,
                       int64_t global_stride, int32_t num_clients, const int64_t* seg_offsets,
                       int32_t nseg, double* seg_sqnorm, void* stream);

/* Per client: total = sqrt(sum_t fl32(sqrt(seg_sqnorm_t))^2) (the reference sums
 * squared per-tensor fp32 norms in double, privacy.py:119-123);
 * clipped = total > max_norm; coef = fl32(max_norm/total);
 * sigma = fl32(min(total,max_norm) * sqrt(2 ln(1.25/delta)) / epsilon) (privacy.py:209). */
int fh_dp_clip_coef(const double* seg_sqnorm, int32_t num_clients, int32_t nseg, double max_norm,
                    double epsilon, double delta, double* total_norm, float* coef,
                    int32_t* clipped, float* sigma, void* stream);

/* out = [global +] ( (clipped ? fl32(delta*coef) : delta) + noise ), each step fp32-rounded.
 * noise = noise_in[z*noise_stride + j] if noise_in != NULL (parity mode: noise drawn by
 * the caller) else sigma[z] * N(0,1) from Philox4x32-10 keyed by (seed, z, j). */
int fh_dp_apply(const float* local, int64_t local_stride, const float* global,
                int64_t global_stride, float* out, int64_t out_stride, int32_t num_clients,
                int64_t P, const float* coef, const int32_t* clipped, const float* sigma,
                const float* noise_in, int64_t noise_stride, uint64_t seed,
                const int64_t* row_ids, void* stream);

/* ---------------- optimizers (torch.optim single-tensor semantics) -------- */
/* SGD(momentum, dampening=0, nesterov=False): buf = first ? g : m*buf + g; p -= lr*buf */
int fh_sgd_step(float* param, const float* grad, float* momentum_buf, int64_t n, float lr,
                float momentum, float weight_decay, int32_t first_step, void* stream);
/* Adam / AdamW (decoupled=1). step_size = lr/(1-beta1^t), bc2_sqrt = sqrt(1-beta2^t),
 * both computed by the caller in double exactly as torch.optim does.  scal_dev
 * (nullable): device float[2] = {bc2_sqrt, -step_size} (fp32-rounded) read at run
 * time instead, so one captured step graph serves every step t. */
int fh_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                 double lr, double beta1, double beta2, double eps, double weight_decay,
                 int32_t decoupled, double step_size, double bc2_sqrt, const float* scal_dev,
                 void* stream);

/* Optimizer steps that finish split weight-gradient reductions (r03).  A convolution's
 * weight gradient split over pixel ranges (fh_conv2d_wgrad_deferred) leaves per-split partial
 * sums; the step sums them as its first operation instead of a separate reduction launch.
 * Rows [0, nclients) of param / grad / state at stride row_stride, row_len floats each
 * (row_len and row_stride multiples of 4, rows 16-B aligned).  Inside each slab range
 * [off, off + len) of a row:  g = sum over s of slab[z][s][j - off], summed in the same
 * order and with the same bits as fh_conv2d_wgrad's own reduction, and g is stored to grad;
 * elsewhere g is read from grad.  Then every element gets the fh_sgd_step / fh_adam_step
 * update (same bits).  slabs: HOST array (copied into the launch) of nslabs <=
 * FH_MAX_GRAD_SLABS ranges, sorted, non-overlapping, off and len multiples of 4, each slab
 * 16-B aligned with client stride splits * len. */
#define FH_MAX_GRAD_SLABS 24
typedef struct {
    int64_t off;       /* first float of the range within a row */
    int64_t len;       /* floats */
    const float* slab; /* device [client][split][len] */
    int32_t splits;
    int32_t reserved;
} fh_grad_slab;
int fh_sgd_step_slabs(float* param, float* grad, float* momentum_buf, int64_t row_stride,
                      int64_t row_len, int32_t nclients, const fh_grad_slab* slabs,
                      int32_t nslabs, float lr, float momentum, float weight_decay,
                      int32_t first_step, void* stream);
int fh_adam_step_slabs(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t row_stride, int64_t row_len, int32_t nclients,
                       const fh_grad_slab* slabs, int32_t nslabs, double lr, double beta1,
                       double beta2, double eps, double weight_decay, int32_t decoupled,
                       double step_size, double bc2_sqrt, const float* scal_dev, void* stream);

/* DP-SGD step (r04): fh_sgd_step_slabs / fh_adam_step_slabs (adam != 0; decoupled = AdamW)
 * for a per-sample-clipped step.  Each slab range holds one split per IMAGE (splits == batch,
 * fh_conv2d_wgrad_persample's slab): g = sum_{i < counts[z]} coef[z][i] * slab[z][i] in image
 * order; then elements [0, n_noise) of every row get g += (sigma_c / counts[z]) * N(0,1) with
 * fh_dpsgd_noise's Philox keys (seed + *seed_dev, philox_row, the row's float4 index); g is
 * stored and the update applied — the bits of fh_persample_slab_wsum + fh_dpsgd_noise + the
 * optimizer step in one launch.  SGD uses lr / momentum / weight_decay / first_step, Adam lr /
 * beta1 / beta2 / eps / weight_decay / step_size / bc2_sqrt / scal_dev as fh_adam_step. */
/* DP-SGD clip coefficients in one launch (r04): for every (client, image < count) the squared
 * norm of that image's gradient over all layers — linear sources by the rank-1 identity
 * ||dy_i||^2 (||x_i||^2 + with_bias) (x [client][batch][in_f], dy [client][batch][out_f]),
 * slab sources (fh_conv2d_wgrad_persample slabs: weights [client][image][per_w], bias behind
 * them at the 256-B aligned offset) as the sum of squares of the image's rows — in fp64, then
 * coef = min(1, max_norm / (count * sqrt(sum))) (the stored gradients are of the batch-mean
 * loss); images >= count get coef 0.  sqnorm (nullable, fp64 [client][batch]) receives the sums.
 * At most 4 sources of each kind.  Replaces fh_linear_persample_sqnorm / fh_persample_slab_sqnorm
 * per layer + fh_dpsgd_clip_coef. */
typedef struct {
    const float* x;
    int64_t x_cs;
    const float* dy;
    int64_t dy_cs;
    int32_t in_f, out_f, with_bias, reserved;
} fh_linear_norm_src;
typedef struct {
    const void* slab;
    int32_t per_w, per_b;
} fh_slab_norm_src;
int fh_dpsgd_norm_clip(const fh_linear_norm_src* lin, int32_t nlin, const fh_slab_norm_src* slabs,
                       int32_t nslab, const int32_t* counts, int32_t nclients, int32_t batch,
                       double max_norm, double* sqnorm, float* coef, void* stream);
/* fh_conv2d_c1_pool_wgrad_persample + fh_dpsgd_norm_clip in ONE launch (r05): each per-image
 * conv1 slab workgroup ends with the image's norm over the sources (which must include this
 * launch's own slab) and its clip coefficient — fh_dpsgd_norm_clip's code and sums.  cout 32. */
int fh_conv2d_c1_pool_wgrad_persample_clip(
    const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs, const uint8_t* idx,
    int64_t i_cs, const float* y, int64_t y_cs, void* slab, size_t slab_bytes,
    const int32_t* counts, int32_t nclients, int32_t batch, int32_t h, int32_t w, int32_t cout,
    int32_t gh, int32_t gw, const fh_linear_norm_src* lin, int32_t nlin,
    const fh_slab_norm_src* slabs, int32_t nslab, double max_norm, double* sqnorm, float* coef,
    void* stream);
/* fh_linear_wgrad on row-scaled dY: dy row b of client z multiplied by rowscale[z][b] as it is
 * loaded (the products fh_scale_rows would store: same bits as scale_rows + linear_wgrad);
 * DP-SGD's clipped linear-layer sums.  batch <= 32, in_f % 32 == 0. */
int fh_linear_wgrad_rowscale(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                             const float* rowscale, float* dw, int64_t dw_cs, float* db,
                             int64_t db_cs, const int32_t* counts, int32_t nclients,
                             int32_t batch, int32_t in_f, int32_t out_f, void* stream);
/* Up to four linear layers' fh_linear_wgrad_rowscale in ONE launch (the same row scales,
 * counts and batch; each layer's tiles, order and bits as its own call): DP-SGD's pass 2 runs
 * fc2's and fc1's clipped sums as one launch (r05).  batch <= 32, in_f % 32 == 0 per layer. */
typedef struct fh_linear_wgrad_src {
    const float* x;
    int64_t x_cs;
    const float* dy;
    int64_t dy_cs;
    float* dw;
    int64_t dw_cs;
    float* db;      /* nullable */
    int64_t db_cs;
    int32_t in_f, out_f;
} fh_linear_wgrad_src;
int fh_linear_wgrad_rowscale_multi(const fh_linear_wgrad_src* layers, int32_t nlayers,
                                   const float* rowscale, const int32_t* counts,
                                   int32_t nclients, int32_t batch, void* stream);
int fh_dpsgd_step_slabs(float* param, float* grad, float* state1, float* state2,
                        int64_t row_stride, int64_t row_len, int32_t nclients,
                        const fh_grad_slab* slabs, int32_t nslabs, const float* coef,
                        const int32_t* counts, int32_t batch, int64_t n_noise, float sigma_c,
                        uint64_t seed, const uint64_t* seed_dev, int32_t adam, double lr,
                        double momentum, double beta1, double beta2, double eps,
                        double weight_decay, int32_t decoupled, int32_t first_step,
                        double step_size, double bc2_sqrt, const float* scal_dev, void* stream);

/* ---------------- convolution / linear (fp32 MFMA implicit GEMM) ----------
 * x: [clients][batch][cin][h][w]; w: [cout][cin][kh][kw] per client; y: [clients][batch][cout][oh][ow].
 * Supported: (kh,kw,stride) in {(3,3,1),(3,3,2),(1,1,1),(1,1,2)}, pad arbitrary. */
/* FWD/DGRAD split K through `workspace` when the output tiling leaves the chip mostly
 * idle (few clients still training); size it with fh_*_workspace (0 = never splits;
 * a NULL / too-small workspace just disables the split). */
size_t fh_conv2d_fwd_workspace(int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w_,
                               int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad);
size_t fh_conv2d_dgrad_workspace(int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                                 int32_t w_, int32_t cout, int32_t kh, int32_t kw, int32_t stride,
                                 int32_t pad);
int fh_conv2d_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs, const float* bias,
                  int64_t b_cs, float* y, int64_t y_cs, const int32_t* counts, int32_t nclients,
                  int32_t batch, int32_t cin, int32_t h, int32_t w_, int32_t cout, int32_t kh,
                  int32_t kw, int32_t stride, int32_t pad, int32_t relu, void* workspace,
                  size_t ws_bytes, void* stream);
/* accumulate = 1: dx += result (residual-branch gradient sums, ResNet shortcut). */
int fh_conv2d_dgrad(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs, float* dx,
                    int64_t dx_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                    int32_t cin, int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                    int32_t stride, int32_t pad, int32_t accumulate, void* workspace,
                    size_t ws_bytes, void* stream);
/* fh_conv2d_dgrad of a 3x3/s1/p1 conv (direct path: square 8/16/32 maps) whose input was
 * relu(BN(bn_x)): stores g = (bn_x*bn_scale + bn_shift > 0) ? dX : 0 and writes the BN
 * backward partials (sum g, sum (bn_x - bn_mean) g) per (client, channel, 256-pixel tile)
 * to bn_part (fh_conv_bnstats_bytes(nclients, batch, cin, h, w_) bytes) for
 * fh_bn_bwd_tiles.  Replaces the reduce pass of fh_bn_bwd (bn.hip bn_bwd_reduce_kernel);
 * pidx non-NULL: a MaxPool2d(2,2) (+ Dropout: pmask / p_drop, pmask NULL = none) sat
 * between the ReLU and this conv; bn_x is then the 2h x 2w map, dX is stored unmasked and
 * the statistics route it to the window argmax (apply pass: fh_bn_bwd_pool_tiles).
 * reference: CIFAR10CNN conv -> bn -> relu (-> pool -> dropout) -> conv,
 * models_pytorch.py:133-150. */
int fh_conv2d_dgrad_bnstats(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs,
                            float* dx, int64_t dx_cs, const float* bn_x, int64_t bnx_cs,
                            const float* bn_scale, const float* bn_shift, int64_t bns_cs,
                            const float* bn_mean, double* bn_part, const uint8_t* pidx,
                            int64_t pi_cs, const uint8_t* pmask, int64_t pm_cs, float p_drop,
                            const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin,
                            int32_t h, int32_t w_, int32_t cout, void* workspace,
                            size_t ws_bytes, void* stream);
/* dw (and db if non-NULL) are overwritten; the conv-bias gradient is folded into the
 * weight-gradient kernel.  workspace >= fh_conv2d_wgrad_workspace(...) bytes. */
size_t fh_conv2d_wgrad_workspace(int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                                 int32_t w_, int32_t cout, int32_t kh, int32_t kw, int32_t stride,
                                 int32_t pad);
int fh_conv2d_wgrad(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs, float* dw,
                    int64_t dw_cs, float* db, int64_t db_cs, void* workspace, size_t ws_bytes,
                    const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin, int32_t h,
                    int32_t w_, int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                    void* stream);

/* Linear: x [clients][batch][in_f], w [out_f][in_f], y [clients][batch][out_f]. */
size_t fh_linear_fwd_workspace(int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f);
size_t fh_linear_dgrad_workspace(int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f);
int fh_linear_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs, const float* bias,
                  int64_t b_cs, float* y, int64_t y_cs, const int32_t* counts, int32_t nclients,
                  int32_t batch, int32_t in_f, int32_t out_f, int32_t relu, void* workspace,
                  size_t ws_bytes, void* stream);
/* fh_linear_fwd followed by fh_dropout_fwd (F.dropout after the layer's ReLU,
 * models_pytorch.py:153-163) as one product: the dropout runs in the forward epilogue
 * with fh_dropout_fwd's keep-mask draws and element order (drop_mode 1 generate / 2 use
 * mask), so y == dropout_fwd(linear_fwd(x)). */
int fh_linear_fwd_dropout(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                          const float* bias, int64_t b_cs, float* y, int64_t y_cs, uint8_t* mask,
                          int64_t m_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                          int32_t in_f, int32_t out_f, int32_t relu, int32_t drop_mode,
                          float p_drop, uint64_t seed, const uint64_t* seed_dev, void* workspace,
                          size_t ws_bytes, void* stream);
int fh_linear_dgrad(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs, float* dx,
                    int64_t dx_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                    int32_t in_f, int32_t out_f, void* workspace, size_t ws_bytes, void* stream);
size_t fh_linear_wgrad_workspace(int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f);
int fh_linear_wgrad(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs, float* dw,
                    int64_t dw_cs, float* db, int64_t db_cs, void* workspace, size_t ws_bytes,
                    const int32_t* counts, int32_t nclients, int32_t batch, int32_t in_f,
                    int32_t out_f, void* stream);
/* One launch for a classifier layer's whole backward (nn.Linear.backward + the
 * F.dropout / ReLU backward of its input, models_pytorch.py:153-163): dw, db (nullable) as
 * fh_linear_wgrad, and dx = (dy W) * keep(mask)/(1-p) where relu_ref > 0 (mask, relu_ref
 * nullable: that factor is skipped).  batch <= 32, in_f % 128 == 0, out_f % 32 == 0, dy
 * rows 16-B aligned; FH_E_UNSUPPORTED otherwise. */
int fh_linear_bwd_fused(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                        const float* w, int64_t w_cs, float* dw, int64_t dw_cs, float* db,
                        int64_t db_cs, float* dx, int64_t dx_cs, const uint8_t* mask,
                        int64_t m_cs, float p_drop, const float* relu_ref, int64_t r_cs,
                        const int32_t* counts, int32_t nclients, int32_t batch, int32_t in_f,
                        int32_t out_f, void* stream);

/*
 * fh_linear_bwd_fused_pool: fh_linear_bwd_fused for a layer whose input x is the flattened
 * output of a 2x2 max-pool over ReLU'd maps [C][OH][OW] (SimpleCNN fc1,
 * models_pytorch.py:91-95 — replaces that layer's backward + the pool's fh_maxpool2_bwd):
 * dX is the gradient of the pool INPUT, planes xh x xw (map 2OH x 2OW top-left), the linear
 * dgrad value routed to the window argmax pidx (dense [C][OH][OW]) where x > 0, zeros at the
 * other window positions; elements outside the map untouched.
 */
int fh_linear_bwd_fused_pool(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                             const float* w, int64_t w_cs, float* dw, int64_t dw_cs, float* db,
                             int64_t db_cs, float* dx, int64_t dx_cs, const uint8_t* pidx,
                             int64_t pi_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                             int32_t C, int32_t OH, int32_t OW, int32_t xh, int32_t xw,
                             int32_t out_f, void* stream);

/* ---------------- BatchNorm2d (+ReLU, +residual add) ----------------------
 * x/y/res: [clients][batch][C][HW]; gamma/beta live in the per-client param
 * rows (stride p_cs); running stats stride r_cs (NULL: not tracked);
 * save_mean/save_invstd: [clients][C].  Train mode: batch statistics over the
 * valid images (fp64 accumulation), running stats momentum-updated with the
 * unbiased variance.  y = relu?( x*alpha + beta' [+ res] ).
 * Each (client, channel) reduction is split over several workgroups; their
 * partials go to `workspace` (>= fh_bn_workspace bytes, shared by train fwd
 * and bwd) and are merged in a fixed order: results are deterministic. */
size_t fh_bn_workspace(int32_t nclients, int32_t batch, int32_t C, int32_t HW);
int fh_bn_fwd_train(const float* x, int64_t x_cs, float* y, int64_t y_cs, const float* res,
                    int64_t res_cs, const float* gamma, const float* beta, int64_t p_cs,
                    float* running_mean, float* running_var, int64_t r_cs, float* save_mean,
                    float* save_invstd, const int32_t* counts, int32_t nclients, int32_t batch,
                    int32_t C, int32_t HW, float eps, float momentum, int32_t relu,
                    void* workspace, size_t ws_bytes, void* stream);
int fh_bn_fwd_eval(const float* x, int64_t x_cs, float* y, int64_t y_cs, const float* res,
                   int64_t res_cs, const float* gamma, const float* beta, int64_t p_cs,
                   const float* running_mean, const float* running_var, int64_t r_cs,
                   const int32_t* counts, int32_t nclients, int32_t batch, int32_t C, int32_t HW,
                   float eps, int32_t relu, void* stream);
/* g = relu ? dy*(yout>0) : dy; dres (nullable) <- g; dgamma/dbeta (stride g_cs) and dx.
 * With relu and yout NULL the mask is recomputed from x (x*alpha + beta' > 0, the
 * forward's own fp32 operations; needs beta, and no residual add before the ReLU). */
int fh_bn_bwd(const float* dy, int64_t dy_cs, const float* yout, int64_t yo_cs, const float* x,
              int64_t x_cs, const float* gamma, const float* beta, int64_t p_cs,
              const float* save_mean,
              const float* save_invstd, float* dx, int64_t dx_cs, float* dres, int64_t dres_cs,
              float* dgamma, float* dbeta, int64_t g_cs, const int32_t* counts, int32_t nclients,
              int32_t batch, int32_t C, int32_t HW, int32_t relu, void* workspace,
              size_t ws_bytes, void* stream);

/* BN backward apply from the partials fh_conv2d_dgrad_bnstats left (g already masked):
 * dgamma / dbeta (stride dg_cs) and dx, as fh_bn_bwd's second pass. */
int fh_bn_bwd_tiles(const double* part, const float* g, int64_t g_cs, const float* x,
                    int64_t x_cs, const float* gamma, int64_t p_cs, const float* save_mean,
                    const float* save_invstd, float* dx, int64_t dx_cs, float* dgamma,
                    float* dbeta, int64_t dg_cs, const int32_t* counts, int32_t nclients,
                    int32_t batch, int32_t C, int32_t HW, void* stream);

/* fh_bn_bwd_pool's apply pass from the partials fh_conv2d_dgrad_bnstats(pidx != NULL)
 * left: dgamma / dbeta and dx (H x W: the BN's map), ReLU mask recomputed from x. */
int fh_bn_bwd_pool_tiles(const double* part, const float* dpool, int64_t dp_cs,
                         const uint8_t* pidx, int64_t pi_cs, const uint8_t* pmask, int64_t pm_cs,
                         float p_drop, const float* x, int64_t x_cs, const float* gamma,
                         const float* beta, int64_t p_cs, const float* save_mean,
                         const float* save_invstd, float* dx, int64_t dx_cs, float* dgamma,
                         float* dbeta, int64_t g_cs, const int32_t* counts, int32_t nclients,
                         int32_t batch, int32_t C, int32_t H, int32_t W, void* stream);

/* BN backward whose upstream gradient comes through MaxPool2d(2,2) (+ the Dropout
 * fused after it, p_drop / pmask as in fh_maxpool2_fwd; pmask NULL = no dropout):
 * the full-resolution gradient is routed from dpool [clients][batch][C][H/2][W/2]
 * by the argmax bytes pidx on the fly (fh_maxpool2_bwd + fh_bn_bwd in one pass pair). */
int fh_bn_bwd_pool(const float* dpool, int64_t dp_cs, const uint8_t* pidx, int64_t pi_cs,
                   const uint8_t* pmask, int64_t pm_cs, float p_drop, const float* yout,
                   int64_t yo_cs, const float* x, int64_t x_cs, const float* gamma,
                   const float* beta, int64_t p_cs, const float* save_mean, const float* save_invstd, float* dx, int64_t dx_cs,
                   float* dgamma, float* dbeta, int64_t g_cs, const int32_t* counts,
                   int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W, int32_t relu,
                   void* workspace, size_t ws_bytes, void* stream);

/* ---------------- DP-SGD: per-sample clipping (north_star extension) -------
 * g = (sum_i min(1, C/||g_i||) g_i + sigma*C*N(0,I)) / B per optimizer step, g_i the
 * gradient of sample i's loss over ALL parameters.  The caller accumulates
 * ||g_i/B||^2 layer by layer into sqnorm [clients][batch] (double; zero it first):
 *   convs   fh_conv2d_persample_sqnorm (per-image WGRAD tiles, workspace query below)
 *   linears fh_linear_persample_sqnorm (||dy_i||^2 (||x_i||^2 + with_bias))
 * then fh_dpsgd_clip_coef -> coef [clients][batch], fh_scale_rows scales each layer's
 * upstream gradient rows by coef before the ordinary WGRAD (clipped sum), and
 * fh_dpsgd_noise adds sigma*C/B * N(0,1) (Philox key seed + seed_dev[0], rows keyed as below).
 * Replaces: nothing in the reference (its DP clips whole update deltas, privacy.py:107-144);
 * sigma follows its Gaussian-mechanism formula (privacy.py:209). */
size_t fh_conv2d_persample_sqnorm_workspace(int32_t nclients, int32_t batch, int32_t cin,
                                            int32_t h, int32_t w, int32_t cout, int32_t kh,
                                            int32_t kw, int32_t stride, int32_t pad);
int fh_conv2d_persample_sqnorm(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                               int32_t with_bias, double* sqnorm, void* workspace,
                               size_t ws_bytes, const int32_t* counts, int32_t nclients,
                               int32_t batch, int32_t cin, int32_t h, int32_t w, int32_t cout,
                               int32_t kh, int32_t kw, int32_t stride, int32_t pad, void* stream);
int fh_linear_persample_sqnorm(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                               int32_t with_bias, double* sqnorm, const int32_t* counts,
                               int32_t nclients, int32_t batch, int32_t in_f, int32_t out_f,
                               void* stream);
/* DP-SGD on the direct kernels (r04): per-image weight-gradient slabs.  A direct WGRAD with one
 * pixel split per image leaves slab [client][image][cout*cin*9] (the gradient of that image's
 * share of the batch-mean loss, g_i / B) and the bias slab [client][image][cout] behind it at a
 * 256-B aligned offset; fh_conv2d_wgrad_persample_workspace gives the slab bytes.
 * fh_conv2d_wgrad_persample: 3x3/s1/p1 on square 8/16/32 maps, channels % 32 (SimpleCNN conv2
 * on its padded 16x16 planes).  fh_conv2d_c1_pool_wgrad_persample: the single-input-channel
 * conv1 from pool1's gradient (fh_conv2d_c1_pool_wgrad's routing), h % 4 == 0.
 * fh_persample_slab_sqnorm: sqnorm[client][image] (fp64, [nclients][batch]) += the image's sum
 * of squares over the slab (weights + bias; per_w % 4 == 0).  fh_persample_slab_wsum: dw =
 * sum_{i < count} coef[client][i] * slab[client][i] in image order (fp32 multiply then add),
 * db likewise from the bias slab (per_b = 0: no bias).  Together they replace the per-sample
 * norm pass and the second WGRAD on coefficient-scaled rows (reference: per-sample clipping is
 * not in the reference; its update clip is privacy.py:107-144, sigma privacy.py:209). */
size_t fh_conv2d_wgrad_persample_workspace(int32_t nclients, int32_t batch, int32_t cin,
                                           int32_t cout);
int fh_conv2d_wgrad_persample(const float* x, int64_t x_cs, const float* dy, int64_t dy_cs,
                              void* slab, size_t slab_bytes, const int32_t* counts,
                              int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w,
                              int32_t cout, void* stream);
int fh_conv2d_c1_pool_wgrad_persample(const float* x, int64_t x_cs, const float* dpool,
                                      int64_t dp_cs, const uint8_t* idx, int64_t i_cs,
                                      const float* y, int64_t y_cs, void* slab, size_t slab_bytes,
                                      const int32_t* counts, int32_t nclients, int32_t batch,
                                      int32_t h, int32_t w, int32_t cout, int32_t gh, int32_t gw,
                                      void* stream);
int fh_persample_slab_sqnorm(const void* slab, int32_t per_w, int32_t per_b,
                             const int32_t* counts, int32_t nclients, int32_t batch,
                             double* sqnorm, void* stream);
int fh_persample_slab_wsum(const void* slab, int32_t per_w, int32_t per_b, const float* coef,
                           const int32_t* counts, int32_t nclients, int32_t batch, float* dw,
                           int64_t dw_cs, float* db, int64_t db_cs, void* stream);
int fh_dpsgd_clip_coef(const double* sqnorm, const int32_t* counts, int32_t nclients,
                       int32_t batch, double max_norm, float* coef, void* stream);
int fh_scale_rows(const float* in, int64_t in_cs, const float* coef, const int32_t* counts,
                  int32_t nclients, int32_t batch, int64_t per_img, float* out, int64_t out_cs,
                  void* stream);
int fh_dpsgd_noise(float* grad, int64_t g_cs, int64_t n, const int32_t* counts, int32_t nclients,
                   int32_t batch, float sigma_c, uint64_t seed, const uint64_t* seed_dev,
                   void* stream);

/* ---------------- MaxPool2d(2,2) (+ fused Dropout after it) ---------------
 * idx: uint8 window argmax [clients][batch][C][H/2][W/2]; drop_mode 0 none,
 * 1 generate keep-mask (Philox4x32-10 keyed by seed, slot, element) into mask,
 * 2 apply the caller's mask (parity).  The Philox key is seed + seed_dev[0]
 * (seed_dev nullable: a per-step device key block for graph replay).  Every seed_dev of
 * this header points to that block, {step key, n_ids, id[0..n_ids)} (uint64): with
 * n_ids != 0 client row z draws under id[z] (its global client id) instead of z, so a
 * client's dropout / augmentation / DP-SGD noise does not depend on its slot.
 * Backward writes all four window slots;
 * xin (nullable) = the pooled ReLU output, to apply the ReLU mask at the argmax. */
int fh_maxpool2_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs, uint8_t* idx,
                    int64_t i_cs, uint8_t* mask, int64_t m_cs, const int32_t* counts,
                    int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                    int32_t drop_mode, float p_drop, uint64_t seed, const uint64_t* seed_dev,
                    void* stream);
int fh_maxpool2_bwd(const float* dy, int64_t dy_cs, const uint8_t* idx, int64_t i_cs,
                    const uint8_t* mask, int64_t m_cs, float p_drop, const float* xin, int64_t x_cs,
                    float* dx, int64_t dx_cs, const int32_t* counts, int32_t nclients,
                    int32_t batch, int32_t C, int32_t H, int32_t W, void* stream);
/* The same pools on H x W maps embedded in the top-left corner of larger planes (SimpleCNN's
 * 14x14 conv runs on 16x16 planes with a zero ring on the direct-conv path): fwd x planes
 * xh x xw and y planes yh x yw; bwd dy planes gh x gw, dx / xin planes xh x xw; idx / mask
 * stay dense [img][C][H/2][W/2].  Nothing outside the map is written. */
int fh_maxpool2_fwd_pitched(const float* x, int64_t x_cs, float* y, int64_t y_cs, uint8_t* idx,
                            int64_t i_cs, uint8_t* mask, int64_t m_cs, const int32_t* counts,
                            int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                            int32_t drop_mode, float p_drop, uint64_t seed,
                            const uint64_t* seed_dev, int32_t xh, int32_t xw, int32_t yh,
                            int32_t yw, void* stream);
int fh_maxpool2_bwd_pitched(const float* dy, int64_t dy_cs, const uint8_t* idx, int64_t i_cs,
                            const uint8_t* mask, int64_t m_cs, float p_drop, const float* xin,
                            int64_t x_cs, float* dx, int64_t dx_cs, const int32_t* counts,
                            int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                            int32_t gh, int32_t gw, int32_t xh, int32_t xw, void* stream);

/* ---------------- Dropout (F.dropout: x * bernoulli(1-p)/(1-p)) ------------
 * drop_mode 1 generate mask (uint8), 2 use the caller's mask.  Backward:
 * dx = dy*mask/(1-p) [* (relu_out > 0)]; mask NULL = ReLU backward only. */
int fh_dropout_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs, uint8_t* mask,
                   int64_t m_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                   int64_t per_img, int32_t drop_mode, float p_drop, uint64_t seed,
                   const uint64_t* seed_dev, void* stream);
int fh_dropout_bwd(const float* dy, int64_t dy_cs, const uint8_t* mask, int64_t m_cs, float p_drop,
                   const float* relu_out, int64_t r_cs, float* dx, int64_t dx_cs,
                   const int32_t* counts, int32_t nclients, int32_t batch, int64_t per_img,
                   void* stream);

/* ---------------- CrossEntropyLoss (mean) fwd+bwd + epoch metrics ---------
 * targets int64 [clients][batch]; dlogits = (softmax - onehot)/count;
 * loss_out[z] = batch mean loss; acc_* (nullable) accumulate the epoch's
 * sum of batch losses, correct argmax predictions and samples seen;
 * reset[z] != 0 (nullable) restarts client z's accumulators (epoch boundary). */
int fh_ce_fwd_bwd(const float* logits, int64_t l_cs, const int64_t* targets, int64_t t_cs,
                  float* dlogits, int64_t d_cs, float* loss_out, double* acc_loss,
                  int64_t* acc_correct, int64_t* acc_seen, const int32_t* reset,
                  const int32_t* counts, int32_t nclients, int32_t batch, int32_t num_classes,
                  void* stream);
/* The classifier head of a training step in one launch per client (replaces the last
 * nn.Linear forward, fh_ce_fwd_bwd, that layer's wgrad / dgrad and the dropout backward in
 * front of it: CIFAR10CNN fc3 models_pytorch.py:159-165, SimpleCNN fc2 :96-97,
 * FederatedResNet fc :241-246, with LocalTrainer's criterion training.py:193-203):
 * logits = x W^T + b (also stored), CE outputs exactly as fh_ce_fwd_bwd, dw / db (nullable),
 * and dx (nullable) = (dlogits W) * keep(mask)/(1-p), zeroed where relu_in and x <= 0.
 * batch <= 32, num_classes <= 128. */
int fh_linear_head_ce(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                      const float* bias, int64_t b_cs, const int64_t* targets, int64_t t_cs,
                      float* logits, int64_t l_cs, float* dlogits, int64_t d_cs, float* loss_out,
                      double* acc_loss, int64_t* acc_correct, int64_t* acc_seen,
                      const int32_t* reset, float* dw, int64_t dw_cs, float* db, int64_t db_cs,
                      float* dx, int64_t dx_cs, const uint8_t* mask, int64_t m_cs, float p_drop,
                      int32_t relu_in, const int32_t* counts, int32_t nclients, int32_t batch,
                      int32_t in_f, int32_t num_classes, void* stream);

/* ---------------- BatchNorm apply + ReLU folded into the consumer (CIFAR10CNN) -------
 * The train-mode BN output relu(x*w*invstd + b - mean*w*invstd) is never written: the
 * statistics pass ends in a per-(client, channel) affine (scale, shift [z][C], stride
 * s_cs) and every consumer of the activation — the next conv's forward and weight
 * gradient, or the 2x2 max-pool — applies relu(x*scale + shift) while loading x.
 * Same fp32 operations as fh_bn_fwd_train's apply pass, so results are bit-identical.
 * (models_pytorch.py:128-137: conv -> bn -> relu -> conv / pool.) */
int fh_bn_fwd_stats(const float* x, int64_t x_cs, const float* gamma, const float* beta,
                    int64_t p_cs, float* running_mean, float* running_var, int64_t r_cs,
                    float* save_mean, float* save_invstd, float* scale_out, float* shift_out,
                    int64_t s_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                    int32_t C, int32_t HW, float eps, float momentum, void* workspace,
                    size_t ws_bytes, void* stream);
/* fh_conv2d_fwd / fh_conv2d_wgrad with x = a BN pre-activation (direct 3x3 path only:
 * 3x3/s1/p1 on 8/16/32 square maps; wgrad also needs cin, cout % 32 == 0; else
 * FH_E_UNSUPPORTED).  Zero padding is applied after the affine (padding of the ReLU
 * output, as in the reference). */
int fh_conv2d_fwd_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                         const float* in_shift, int64_t aff_cs, const float* w, int64_t w_cs,
                         const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                         const int32_t* counts, int32_t nclients, int32_t batch, int32_t cin,
                         int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                         int32_t stride, int32_t pad, int32_t relu, void* workspace,
                         size_t ws_bytes, void* stream);
int fh_conv2d_wgrad_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                           const float* in_shift, int64_t aff_cs, const float* dy, int64_t dy_cs,
                           float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* workspace,
                           size_t ws_bytes, const int32_t* counts, int32_t nclients,
                           int32_t batch, int32_t cin, int32_t h, int32_t w_, int32_t cout,
                           int32_t kh, int32_t kw, int32_t stride, int32_t pad, void* stream);
/* fh_conv2d_wgrad (in_scale / in_shift NULL) or fh_conv2d_wgrad_bnrelu without the final
 * reduction: when the kernel leaves partial sums (*splits_out >= 1 of them) they stay in `slab`
 * (sized by fh_conv2d_wgrad_workspace) — weights [client][split][cout*cin*kh*kw] at byte 0,
 * bias [client][split][cout] at byte *bias_off_out — for an optimizer step to finish
 * (fh_sgd_step_slabs / fh_adam_step_slabs; a one-split slab is copied by it);
 * *splits_out == 0: dw / db written directly.  (r06: one-split slab plans — single-channel,
 * small-cin and stride-2 kernels — used to report 1, read as "written directly", so that
 * layer's gradient was dropped; found by tests/test_full_plan_resnet_gpu.py, K5.) */
int fh_conv2d_wgrad_deferred(const float* x, int64_t x_cs, const float* in_scale,
                             const float* in_shift, int64_t aff_cs, const float* dy,
                             int64_t dy_cs, float* dw, int64_t dw_cs, float* db, int64_t db_cs,
                             void* slab, size_t slab_bytes, const int32_t* counts,
                             int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w_,
                             int32_t cout, int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                             int32_t* splits_out, int64_t* bias_off_out, void* stream);
int fh_maxpool2_fwd_bnrelu(const float* x, int64_t x_cs, const float* in_scale,
                           const float* in_shift, int64_t aff_cs, float* y, int64_t y_cs,
                           uint8_t* idx, int64_t i_cs, uint8_t* mask, int64_t m_cs,
                           const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                           int32_t H, int32_t W, int32_t drop_mode, float p_drop, uint64_t seed,
                           const uint64_t* seed_dev, void* stream);
/* BatchNorm statistics from the producing convolution (models_pytorch.py:128-137 conv ->
 * bn; replaces the statistics pass of nn.BatchNorm2d's train forward): the direct-conv
 * forward (fh_conv2d_fwd_bnrelu semantics, in_scale/in_shift nullable, no ReLU on y) also
 * writes one fp64 (sum of y, sum of y^2) pair per (client, channel, 256-pixel tile of the
 * client's [batch*H*W] pixels) into bn_part (fh_conv_bnstats_bytes; tiles past a client's
 * count are zero), and fh_bn_finalize_tiles merges them in tile order into fh_bn_fwd_stats'
 * outputs — y is never re-read for its statistics. */
size_t fh_conv_bnstats_bytes(int32_t nclients, int32_t batch, int32_t cout, int32_t h,
                             int32_t w_);
int fh_conv2d_fwd_bnstats(const float* x, int64_t x_cs, const float* in_scale,
                          const float* in_shift, int64_t aff_cs, const float* w, int64_t w_cs,
                          const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                          double* bn_part, const int32_t* counts, int32_t nclients,
                          int32_t batch, int32_t cin, int32_t h, int32_t w_, int32_t cout,
                          void* workspace, size_t ws_bytes, void* stream);
/* conv (3x3 / s1 / p1, bias) -> ReLU -> 2x2 max-pool of the top-left pool_hw x pool_hw map of
 * each h x w plane (h = w = 8 or 16): SimpleCNN conv2 -> relu -> pool2 on the 16x16 planes that
 * hold its 14x14 map (replaces conv2d_fwd + maxpool2_fwd of models_pytorch.py:88-89).  py /
 * pidx: dense [img][cout][pool_hw/2][pool_hw/2], the values and first-max argmax of
 * fh_maxpool2_fwd_pitched bit for bit: pooled in the conv's epilogue (unsplit launches) or in
 * the split-K reduction (16x16 planes).  y (h x w planes) is scratch, written only by split
 * launches on 8x8 planes (pooled by a separate pass); the pool's backward takes its ReLU mask
 * from py (fh_maxpool2_bwd_ymask). */
int fh_conv2d_fwd_relu_pool(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                            const float* bias, int64_t b_cs, float* y, int64_t y_cs, float* py,
                            int64_t py_cs, uint8_t* pidx, int64_t pi_cs, const int32_t* counts,
                            int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w_,
                            int32_t cout, int32_t pool_hw, void* workspace, size_t ws_bytes,
                            void* stream);
/* fh_bn_finalize_tiles fused into the 2x2 max-pool (+dropout, drop_mode as fh_maxpool2_fwd)
 * of the BN-ReLU output (CIFAR10CNN conv -> bn -> relu -> pool -> dropout,
 * models_pytorch.py:139-155): the same outputs as fh_bn_finalize_tiles followed by
 * fh_maxpool2_fwd_bnrelu, one launch. */
int fh_maxpool2_fwd_bnfinalize(const double* part, const float* gamma, const float* beta,
                               int64_t p_cs, float* running_mean, float* running_var,
                               int64_t r_cs, float* save_mean, float* save_invstd,
                               float* scale_out, float* shift_out, int64_t s_cs, const float* x,
                               int64_t x_cs, float* y, int64_t y_cs, uint8_t* idx, int64_t i_cs,
                               uint8_t* mask, int64_t m_cs, const int32_t* counts,
                               int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                               float eps, float momentum, int32_t drop_mode, float p_drop,
                               uint64_t seed, const uint64_t* seed_dev, void* stream);
int fh_bn_finalize_tiles(const double* part, const float* gamma, const float* beta,
                         int64_t p_cs, float* running_mean, float* running_var, int64_t r_cs,
                         float* save_mean, float* save_invstd, float* scale_out,
                         float* shift_out, int64_t s_cs, const int32_t* counts,
                         int32_t nclients, int32_t batch, int32_t C, int32_t HW, float eps,
                         float momentum, void* stream);
/* The input gradient of a ResNet down-sampling block in one launch (models_pytorch.py:176-194:
 * conv1 3x3/s2/p1 and the 1x1/s2 projection shortcut read the same input):
 * dx (=|+=) dgrad_3x3s2(dy, w) + dgrad_1x1s2(dy_sc, w_sc); dy_sc has dy's shape, w_sc is
 * [cout][cin] per client.  Replaces the two fh_conv2d_dgrad calls (the second accumulating).
 * Direct stride-2 kernel only (square 32/16 maps, cin % 32 == 0, cout % 8 == 0, aligned
 * rows): FH_E_UNSUPPORTED otherwise.  Workspace: fh_conv2d_dgrad_workspace of the 3x3. */
int fh_conv2d_dgrad_s2_shortcut(const float* dy, int64_t dy_cs, const float* w, int64_t w_cs,
                                const float* dy_sc, int64_t dysc_cs, const float* w_sc,
                                int64_t wsc_cs, float* dx, int64_t dx_cs, const int32_t* counts,
                                int32_t nclients, int32_t batch, int32_t cin, int32_t h, int32_t w_,
                                int32_t cout, int32_t accumulate, void* workspace, size_t ws_bytes,
                                void* stream);
/* SimpleCNN conv1 -> ReLU -> 2x2 max-pool (models_pytorch.py:80-82) in one launch: cin = 1,
 * 3x3/s1/p1, cout 32 or 64; y = the pooled output in planes yh x yw (map in the top-left
 * corner), idx the dense uint8 window argmax; the same values as fh_conv2d_fwd(relu=1) +
 * fh_maxpool2_fwd, the full-resolution ReLU output never written. */
int fh_conv2d_c1_pool_fwd(const float* x, int64_t x_cs, const float* w, int64_t w_cs,
                          const float* bias, int64_t b_cs, float* y, int64_t y_cs, uint8_t* idx,
                          int64_t i_cs, const int32_t* counts, int32_t nclients, int32_t batch,
                          int32_t h, int32_t w_, int32_t cout, int32_t yh, int32_t yw,
                          void* stream);
/* fh_conv2d_c1_pool_fwd with the step's batch gather folded in (r04): x [client][batch][h][w]
 * is WRITTEN from the raw uint8 images data[gidx[client][b]] ([N][h][w], one channel) with
 * fh_gather_u8's normalisation (x = (u / 255 - mean) / std; no crop / flip) and
 * y_lab[client][b] = labels[gidx[client][b]] — fh_gather_u8's x and labels bit for bit — and
 * the pooled output / argmax as fh_conv2d_c1_pool_fwd on that x.  Replaces gather +
 * conv1 -> relu -> pool1 of SimpleCNN's training step (data_loader.py:298-301,
 * models_pytorch.py:86-87). */
int fh_conv2d_c1_pool_fwd_u8(const uint8_t* data, const int64_t* labels, const int64_t* gidx,
                             int64_t g_cs, float mean, float stdv, float* x, int64_t x_cs,
                             int64_t* y_lab, int64_t yl_cs, const float* w, int64_t w_cs,
                             const float* bias, int64_t b_cs, float* y, int64_t y_cs,
                             uint8_t* idx, int64_t i_cs, const int32_t* counts, int32_t nclients,
                             int32_t batch, int32_t h, int32_t w_, int32_t cout, int32_t yh,
                             int32_t yw, void* stream);
/* fh_maxpool2_bwd (pitched planes: dy / y gh x gw, dx xh x xw) with the ReLU mask at the
 * argmax taken from the pooled output y (> 0), for a forward that never wrote the
 * full-resolution ReLU output (fh_conv2d_c1_pool_fwd); no dropout. */
int fh_maxpool2_bwd_ymask(const float* dy, int64_t dy_cs, const uint8_t* idx, int64_t i_cs,
                          const float* y, int64_t y_cs, float* dx, int64_t dx_cs,
                          const int32_t* counts, int32_t nclients, int32_t batch, int32_t C,
                          int32_t H, int32_t W, int32_t gh, int32_t gw, int32_t xh, int32_t xw,
                          void* stream);
/* Its weight gradient: fh_maxpool2_bwd(dpool, idx, xin = ReLU output) + fh_conv2d_wgrad in
 * one pass (the ReLU mask at the argmax is y > 0); dpool / y in planes gh x gw.  Workspace:
 * fh_conv2d_wgrad_workspace(nclients, batch, 1, h, w, cout, 3, 3, 1, 1). */
int fh_conv2d_c1_pool_wgrad(const float* x, int64_t x_cs, const float* dpool, int64_t dp_cs,
                            const uint8_t* idx, int64_t i_cs, const float* y, int64_t y_cs,
                            float* dw, int64_t dw_cs, float* db, int64_t db_cs, void* workspace,
                            size_t ws_bytes, const int32_t* counts, int32_t nclients,
                            int32_t batch, int32_t h, int32_t w_, int32_t cout, int32_t gh,
                            int32_t gw, void* stream);
/* fh_conv2d_c1_pool_wgrad without the final reduction (as fh_conv2d_wgrad_deferred): the
 * *splits_out >= 1 per-chunk partials stay in `slab` for fh_sgd_step_slabs /
 * fh_adam_step_slabs. */
int fh_conv2d_c1_pool_wgrad_deferred(const float* x, int64_t x_cs, const float* dpool,
                                     int64_t dp_cs, const uint8_t* idx, int64_t i_cs,
                                     const float* y, int64_t y_cs, float* dw, int64_t dw_cs,
                                     float* db, int64_t db_cs, void* slab, size_t slab_bytes,
                                     const int32_t* counts, int32_t nclients, int32_t batch,
                                     int32_t h, int32_t w_, int32_t cout, int32_t gh, int32_t gw,
                                     int32_t* splits_out, int64_t* bias_off_out, void* stream);
/* fh_bn_fwd_train (its apply pass: y = [relu](bn(x) [+ res]), save_mean / save_invstd,
 * running statistics) from the tiles fh_conv2d_fwd_bnstats left — FederatedResNet's stem
 * bn1 and block bn2 + residual + ReLU (models_pytorch.py:189-194, :241-242), whose output the
 * next block reads twice and is therefore materialised. */
int fh_bn_apply_tiles(const double* part, const float* x, int64_t x_cs, float* y, int64_t y_cs,
                      const float* res, int64_t res_cs, const float* gamma, const float* beta,
                      int64_t p_cs, float* running_mean, float* running_var, int64_t r_cs,
                      float* save_mean, float* save_invstd, const int32_t* counts,
                      int32_t nclients, int32_t batch, int32_t C, int32_t HW, float eps,
                      float momentum, int32_t relu, void* stream);

/* ---------------- launch planning ---------------------------------------------
 * Share of the chip (0, 1] that the split-K planners of the conv / linear entry points
 * aim to fill, for launches issued by the CALLING THREAD (thread-local; default 1).
 * A client lane running concurrently with others asks for less (fedhip/lanes.py). */
int fh_set_fill_fraction(float fraction);
float fh_get_fill_fraction(void);

/* Dual-role layer backward (CIFAR10CNN / ResNet 3x3 layers, the WGRAD + DGRAD pair of
 * models_pytorch.py's autograd backward).  mode 1 or 2 arms the CALLING THREAD's next
 * fh_conv2d_wgrad* call: a direct quadrant-wave WGRAD whose dW needs no reduction launch is
 * held and issued in one grid with the next direct DGRAD on the same stream (1: WGRAD
 * workgroups first, 2: DGRAD first), else on its own before it.  mode 0 issues anything still
 * held and disarms; call it after the pair's DGRAD.  mode -1 disarms and drops a held launch
 * unissued (a caller's error path). */
int fh_conv_pair(int32_t mode);
/* The calling thread's pairing state, for instrumentation (bench.py's per-launch timing
 * attributes a dual launch to both roles' work): *held = 1 while a WGRAD launch is held for
 * the next DGRAD, *dual_launches = dual-role grids this thread has issued so far. */
int fh_conv_pair_status(int32_t* held, int64_t* dual_launches);
/* r05: fh_conv_defer_dgrad(1) arms the calling thread's next split direct DGRAD on 16x16
 * planes with a plain sum epilogue to leave its partials unreduced; the conv1 weight gradient
 * that reads its output (fh_conv2d_c1_pool_wgrad[_deferred], fh_conv2d_c1_pool_wgrad_persample
 * [_clip]) sums them while staging (the epilogue's order: the same bits).  Any other consumer
 * path, or fh_conv_defer_dgrad(0), launches the skipped reduction first. */
int fh_conv_defer_dgrad(int32_t on);
/* r06 (instrumentation): DGRADs the calling thread left unreduced under fh_conv_defer_dgrad, and
 * how many of those partial slabs a conv1 weight-gradient consumer summed while staging. */
int fh_conv_defer_status(int64_t* deferred, int64_t* taken);
/* r06: fh_conv_bn_defer(max_elems) arms the calling thread's next fh_conv2d_fwd_bnstats /
 * fh_conv2d_dgrad_bnstats call: when it plans a split direct launch (at most 4 splits, batch x
 * plane <= min(max_elems, 8192)), its split reduction — the splitk_epilogue launch that writes
 * the output and the statistics tiles — is left to the BatchNorm call that consumes those tiles, which the
 * caller issues next: fh_bn_finalize_tiles or fh_maxpool2_fwd_bnfinalize after the FWD,
 * fh_bn_bwd_tiles or fh_bn_bwd_pool_tiles after the DGRAD.  That call then runs the reduction
 * and its own pass as ONE launch (one workgroup per channel and client), every stored value
 * bit-identical to the two launches; the DGRAD's own output (the masked or pooled gradient,
 * read by nothing but that BN call) is then not written.  Any other library call that finds
 * the reduction pending launches it first; fh_conv_pair(-1) drops it.  max_elems 0 disarms.
 * Measured no faster than the two launches on MI355X (fedhip.ops.SPLIT_BN: off by default).
 * Replaces nothing in the reference: the pair is BatchNorm2d after Conv2d,
 * src/shared/models_pytorch.py:133-150 (CIFAR10CNN), :189-194 (FederatedResNet block). */
int fh_conv_bn_defer(int32_t max_elems);
/* r06 (instrumentation): split reductions the calling thread left to a BN call, and fused
 * launches the BN calls issued. */
int fh_conv_bn_defer_status(int64_t* deferred, int64_t* taken);
/* r06: in-launch split-K reduction.  A direct 3x3 FWD / DGRAD (and the DGRAD role of the
 * dual-role backward) whose plan splits the input-channel reduction stores each split's partial
 * tile write-through and takes a ticket; the tile's last arriving workgroup sums the partials in
 * split order and runs the unsplit epilogue (bias, ReLU, BN statistics, pool) — no
 * splitk_epilogue launch.  `tickets` = n uint32 counters (one per output tile of a launch),
 * zeroed ONCE by the caller, kept alive while launches or captured steps that used them may run,
 * and left zero by every launch; per calling thread (one buffer per stream: concurrent launches
 * must not share counters).  NULL / 0 = split-K epilogue launches as before. */
int fh_set_split_tickets(void* tickets, int64_t n);
/* launches of the calling thread that reduced their split-K in-launch (instrumentation) */
int fh_split_tickets_status(int64_t* inl_launches);
/* The next WGRAD + DGRAD pair's output gradient is a 2x2 max-pool's backward (SimpleCNN conv2,
 * models_pytorch.py:88-90, pool2 after relu(conv2)): dY(y, x) = dpool[y/2][x/2] where (y, x) is
 * the window's argmax pidx and the pooled ReLU output ypool there is > 0, else 0
 * (fh_maxpool2_bwd_ymask), pooled planes ph x ph, dense.  Call after fh_conv_pair(mode).  When
 * the pair becomes one dual-role launch on 16x16 planes both roles route dY on load and the
 * pair's dY tensor is never written; otherwise the library first fills it with
 * fh_maxpool2_bwd_ymask.  fh_conv_pair(0 / -1) disarms. */
int fh_conv_pooled_dy(const float* dpool, int64_t dp_cs, const uint8_t* pidx, int64_t pi_cs,
                      const float* ypool, int64_t yp_cs, int32_t ph);

/* Lane streams (fedhip/lanes.py; replaces the reference's one-thread-per-client
 * concurrency, federated_simulation.py:309-318).  cu_mask (nullable; mask_words 32-bit
 * words, bit i = CU i) restricts the stream to those CUs (hipExtStreamCreateWithCUMask);
 * otherwise the stream gets dispatch priority `priority` (lower = higher, HIP's range).
 * *stream_out is a hipStream_t; release it with fh_stream_destroy. */
int fh_stream_create(int32_t priority, const uint32_t* cu_mask, int32_t mask_words,
                     void** stream_out);
int fh_stream_destroy(void* stream);

/* Step programs (csrc/program.hip; replaces torch.cuda.CUDAGraph.replay for concurrent
 * lanes: +1.3 % on KT).  fh_record_begin makes this thread's libfedhip launches ALSO append
 * to a new program (kernel, geometry, LDS bytes and a private copy of the arguments);
 * fh_record_end stops it.  fh_program_launch re-issues the list on `stream`.  A program
 * owns everything it launches with except the device buffers its arguments point at.
 * fh_graph_node_counts: kernel / non-kernel work nodes of a captured hipGraph_t, so the
 * caller can verify a recording made during that capture saw the whole step. */
int fh_record_begin(void** program_out);
int fh_record_end(void* program, int32_t* kernels_out);
int fh_graph_node_counts(void* graph, int32_t* kernels_out, int32_t* others_out);

/*
 * fh_program_matches_graph: *match_out = 1 when `program` (fh_record_begin/end) is a faithful
 * copy of the captured hipGraph_t `graph`: no non-kernel work node in the graph, and the
 * graph's kernel functions equal the recorded ones as multisets.  0 otherwise (the caller
 * replays the graph).  Stronger than comparing fh_graph_node_counts with the recorded count.
 */
int fh_program_matches_graph(void* program, void* graph, int32_t* match_out);
int fh_program_launch(void* program, void* stream);
/* r06: relocation of the per-step input slot.  fh_program_relocate marks every 8-byte
 * argument word of the recorded launches (struct fields included) equal to one of ptrs[0..n),
 * each inside [base, base + len) — the step's per-step input slot and its views; *found = the
 * number of words, or -1 when some other word points into the slot (then only
 * fh_program_launch is valid).  fh_program_launch_at rewrites those words to the same offsets
 * from new_base (another row laid out like the slot) and issues the program: the step reads
 * its inputs in place, without a copy into the slot first. */
int fh_program_relocate(void* program, const uint64_t* ptrs, int32_t nptrs, uint64_t base,
                        int64_t len, int32_t* found);
int fh_program_launch_at(void* program, void* stream, uint64_t new_base);
int fh_program_destroy(void* program);

/* Launch timestamps of the dual-role conv backward (bench.py's roofline over the TIMED
 * rounds; replaces the reference's wall-clock timers around train_local_model,
 * training.py:86,140).  While rec is non-null, every dconv_wgrad_dual_kernel launch of the
 * layer shape (map w x w, cin -> cout) appends one record per workgroup to rec [cap][4]
 * uint32: its dispatch packet key, the shape key, and the workgroup's first / last wall-clock
 * tick (100 MHz counter, low 32 bits; fh_wall_clock_khz); *count (uint32, caller-zeroed) is
 * the next free record.  A launch's duration is max(last) - min(first) over its records —
 * the kernel trace's begin-to-end.  rec = null turns it off.  Host calls, outside a capture. */
int fh_launch_ts_set(void* rec, void* count, uint32_t cap, int32_t w, int32_t cin, int32_t cout);
int fh_wall_clock_khz(int32_t* khz);
/* dst[0:nbytes) = src[0:nbytes) by a kernel (16-B aligned, nbytes % 16 == 0): the per-step
 * input row copy of a lane in program mode. */
int fh_copy_bytes(const void* src, void* dst, int64_t nbytes, void* stream);

/* ---------------- on-device input pipeline (data_loader.py:298-301, 454-458) -----
 * x[z][b] = Normalize(RandomHorizontalFlip(RandomCrop(data[idx[z][b]], pad)))
 * from raw uint8 HWC images (torchvision layout) to fp32 NCHW: (u/255 - mean_c) /
 * std_c (mean/stdv: HOST float[C], C <= 4); pad 0 = no crop, flip 0 = no flip.
 * Crop/flip per image from aug_in (uchar4 {i, j, flip, -} per [z][b], stride
 * aug_cs; replay) or Philox(seed + *seed_dev, (z, b)), then recorded to aug_out
 * (nullable).  y[z][b] = labels[idx[z][b]] (y nullable). */
int fh_gather_u8(const uint8_t* data, const int64_t* labels, const int64_t* idx, int64_t idx_cs,
                 float* x, int64_t x_cs, int64_t* y, int64_t y_cs, const int32_t* counts,
                 int32_t nclients, int32_t batch, int32_t C, int32_t H, int32_t W,
                 const float* mean, const float* stdv, int32_t pad, int32_t flip,
                 const uint8_t* aug_in, uint8_t* aug_out, int64_t aug_cs, uint64_t seed,
                 const uint64_t* seed_dev, void* stream);

/* ---------------- update compression (compression.py:123-368) -----
 * Per client row z and parameter segment s = [seg_offsets[s], seg_offsets[s+1]):
 * v = x[z] - base[z] (base nullable: v = x[z]; base_cs 0 broadcasts one row) and
 * out[z] = base[z] + decompress(compress(v)) (out nullable; may alias x).
 * Segments are processed in chunks of fh_compress_chunk_elems() elements;
 * chunk_offsets[s] (device int32[nseg+1]) = cumulative ceil(len_s / chunk), nchunks =
 * chunk_offsets[nseg].
 *
 * fh_quantize_rows   QuantizationCompressor._quantize_tensor + _dequantize_tensor
 *                    (:203-244), bits in [1,16]; codes (nullable, bits <= 8) get the
 *                    uint8 wire codes; scale_out / zp_out (nullable, [C][nseg]) the
 *                    per-segment scale (double) and zero point.  Asymmetric mode on a
 *                    constant segment raises in the reference (round(inf)); here that
 *                    segment passes through unchanged and zp_out = INT64_MIN.
 * fh_topk_rows       TopKSparsificationCompressor._sparsify_tensor + _desparsify_tensor
 *                    (:327-365) with k = seg_k[s] (device int64[nseg]); keep (nullable)
 *                    gets the uint8 keep-mask.  Ties at the k-th magnitude: lowest
 *                    flat indices are kept. */
int64_t fh_compress_chunk_elems(void);
int64_t fh_quantize_workspace(int32_t nclients, int32_t nchunks);
int fh_quantize_rows(const float* x, int64_t x_cs, const float* base, int64_t base_cs, float* out,
                     int64_t out_cs, uint8_t* codes, int64_t codes_cs, int32_t nclients,
                     const int64_t* seg_offsets, const int32_t* chunk_offsets, int32_t nseg,
                     int32_t nchunks, int32_t bits, int32_t symmetric, double* scale_out,
                     int64_t* zp_out, void* ws, size_t ws_bytes, void* stream);
int64_t fh_topk_workspace(int32_t nclients, int32_t nseg, int32_t nchunks);
int fh_topk_rows(const float* x, int64_t x_cs, const float* base, int64_t base_cs, float* out,
                 int64_t out_cs, uint8_t* keep, int64_t keep_cs, int32_t nclients,
                 const int64_t* seg_offsets, const int32_t* chunk_offsets, const int64_t* seg_k,
                 int32_t nseg, int32_t nchunks, void* ws, size_t ws_bytes, void* stream);

/* ---------------- evaluation metrics (training.py:214-242, 307-360) ----------
 * Eval-mode metrics of [nclients][batch][K] logits: per image the first-index
 * argmax (torch.max) and the CE loss.  loss_sum[z] += sum of the slot's image
 * losses (fp64) and correct[z] += its correct predictions (both nullable,
 * accumulated across calls); class_correct[k] / class_total[k] (nullable
 * together) count correct and seen images of label k (integer atomics). */
int fh_eval_metrics(const float* logits, int64_t l_cs, const int64_t* targets, int64_t t_cs,
                    const int32_t* counts, int32_t nclients, int32_t batch, int32_t num_classes,
                    double* loss_sum, int64_t* correct, int64_t* class_correct,
                    int64_t* class_total, void* stream);

/* ---------------- AdaptiveAvgPool2d((1,1)) --------------------------------- */
int fh_avgpool_fwd(const float* x, int64_t x_cs, float* y, int64_t y_cs, const int32_t* counts,
                   int32_t nclients, int32_t batch, int32_t C, int32_t HW, void* stream);
int fh_avgpool_bwd(const float* dy, int64_t dy_cs, float* dx, int64_t dx_cs,
                   const int32_t* counts, int32_t nclients, int32_t batch, int32_t C, int32_t HW,
                   void* stream);

/* ---------------- on-device batch assembly (DataLoader replacement) -------
 * x[z][b] = data[idx[z*idx_cs+b]], y[z][b] = labels[idx[..]] for b < counts[z]. */
int fh_gather_batch(const float* data, const int64_t* labels, const int64_t* idx, int64_t idx_cs,
                    float* x, int64_t x_cs, int64_t* y, int64_t y_cs, int64_t sample_elems,
                    const int32_t* counts, int32_t nclients, int32_t batch, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FEDHIP_H_ */
