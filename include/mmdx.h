/*
 * mmdx — MI355X-native (gfx950) kernels for the multimodal diagnosis hot path of
 * PravCoder/Multi-Modal-Medical-Imaging-and-Report-ML-Diagnosis-System.
 *
 * C ABI of libmmdx_hip.so.  Plain pointers and sizes only; every buffer is owned by the
 * caller (PyTorch's caching allocator in the shipped host code); the library never
 * allocates or frees caller memory.  Where a call needs scratch, the caller queries
 * `*_workspace_size` and passes a buffer of at least that many bytes.
 *
 * The reference has no native code and no FFI: its hot path is pure PyTorch-CPU
 * (backend/ml/pipelines/training_pipeline.py, "TP" below).  Each entry point names the
 * reference operator it replaces; the Python host layer (mmdx.training_pipeline) keeps
 * the reference's class/function surface and binds these symbols with ctypes.
 *
 * Conventions
 *   dtype:      0 = fp32 (parity path, exact-f32 MFMA), 1 = bf16 (throughput path),
 *               2 = fp16 (C5's "fp16 MFMA": dense GEMM, attention, LayerNorm, text / ViT
 *               kernels; the ResNet and BiLSTM entry points reject it)
 *   images:     NHWC, channels innermost; conv weights packed [Cout][R][S][Cin] ("KRSC")
 *               for fwd and [Cin][R][S][Cout] ("CRSK") for dgrad; fp32 master weights
 *               and gradients stay in PyTorch's [Cout][Cin][R][S] ("KCRS") layout.
 *   matrices:   row-major; "kmajor" = the contraction index is the contiguous one.
 *   stream:     a hipStream_t passed as void*; every call is stream-ordered, reentrant,
 *               graph-capturable (no allocation, no sync, no host readback).
 *   return:     0 on success, negative errno / -hipError_t on failure;
 *               mmdx_last_error() gives a thread-local message.
 */
#ifndef MMDX_H_
#define MMDX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { MMDX_F32 = 0, MMDX_BF16 = 1, MMDX_F16 = 2 };
enum { MMDX_ACT_NONE = 0, MMDX_ACT_RELU = 1, MMDX_ACT_GELU = 2, MMDX_ACT_GELU_BWD = 3 };

int mmdx_version(void);
const char* mmdx_last_error(void);
/* Re-read the MMDX_* launch-heuristic environment knobs (tile / split choices; read once per
 * process otherwise).  For tests and A/B runs that switch a knob between launches; not to be
 * called while another thread issues launches. */
int mmdx_reload_config(void);
/* A non-blocking HIP stream on `cus` of the device's compute units (evenly spread; 0 = all)
 * with the given priority (cus < all: hipExtStreamCreateWithCUMask, default priority).  Used
 * for the trunk's weight-gradient stream (MMDX_WGRAD_CUS).  *out: the hipStream_t. */
int mmdx_stream_create(int priority, int cus, void** out);
int mmdx_stream_destroy(void* stream);

/* ---------------------------------------------------------------- GEMM (nn.Linear)
 * C[M,N] = act(alpha * sum_k A(m,k) B(n,k) + bias[n] + addend[m,n]) + beta * C
 * (addend: optional fp32, leading dim ldc — lets a concat-input Linear run as two GEMMs)
 * A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m];  same for B with (n,k).
 * c_dtype may differ from dtype (bf16 compute -> fp32 weight-gradient output).
 * preact (optional, c_dtype, ld = ldc) receives alpha*acc + bias before the activation.
 * act = MMDX_ACT_GELU_BWD: preact is an INPUT (the forward's pre-activation, read, not
 * written) and C = alpha*acc * gelu'(preact) (+ beta*C): the GELU backward fused into the
 * GEMM that produces the post-activation gradient (BERT / ViT FFN, fusion MLP).
 * Replaces: nn.Linear fwd/bwd in ImageEncoderCNN.proj/classifier (TP:189,194),
 * TextEncoderTransformer.proj/classifier (TP:365,367), BERT dense layers (TP:360 ->
 * transformers BertModel), fusion_mlp[0] + GELU (TP:534-536), disease_head (TP:542). */
size_t mmdx_gemm_workspace_size(int dtype, int M, int N, int K);
/* mmdx_gemm plus a residual [M][ldc] of C's dtype added last (after the activation and
 * beta*C): C = act(alpha*A B^T + bias) + beta*C + residual; residual must not alias C.
 * Replaces: the residual adds of torchvision's EncoderBlock (x + mlp(ln_2(x)), vit_b_16). */
int mmdx_gemm_res(int dtype, int M, int N, int K, const void* A, long lda, int a_kmajor,
                  const void* B, long ldb, int b_kmajor, void* C, long ldc, int c_dtype,
                  const float* bias, const float* addend, int act, float alpha, float beta,
                  void* preact, const void* residual, void* workspace, size_t ws_bytes,
                  void* stream);
/* Weight gradient of a Linear layer with its bias gradient: C = A B for A = dY^T and B = X
 * both R-major (element (m, k) of A at A[k*lda + m]: dY [K tokens][lda]), alpha 1, beta 0,
 * and db[m] = sum_k A(m, k) (the column sums of dY) — for 16-bit split-K problems computed by
 * the GEMM blocks of column tile 0 from their own A fragments (one extra MFMA per fragment
 * against a ones operand) and reduced over the splits, so dY is not read again; otherwise
 * (fp32, unsplit grids, unaligned operands, MMDX_WGRAD_BIAS_FUSED=0) mmdx_gemm followed by
 * mmdx_bias_grad (needs lda == M).
 * Replaces: the weight and bias gradients of nn.Linear in the BERT / ViT layers (TP:360). */
size_t mmdx_gemm_bias_grad_workspace_size(int dtype, int M, int N, int K);
int mmdx_gemm_bias_grad(int dtype, int M, int N, int K, const void* A, long lda, const void* B,
                        long ldb, void* C, long ldc, int c_dtype, float* db, void* workspace,
                        size_t ws_bytes, void* stream);
int mmdx_gemm(int dtype, int M, int N, int K,
              const void* A, long lda, int a_kmajor,
              const void* B, long ldb, int b_kmajor,
              void* C, long ldc, int c_dtype,
              const float* bias, const float* addend, int act, float alpha, float beta,
              void* preact, void* workspace, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- convolution
 * Replaces: every nn.Conv2d of torchvision resnet18/50 reached through
 * ImageEncoderCNN._backbone_forward_grad/_nograd (TP:279-289, TP:183). */
typedef struct {
  int N, H, W, C;      /* input NHWC */
  int K;               /* output channels */
  int R, S;            /* filter height, width */
  int stride_h, stride_w, pad_h, pad_w;
  int P, Q;            /* output height, width */
} mmdx_conv_desc;

/* fp32 KCRS master -> packed compute-dtype copies (either output may be NULL).
 * Channel padding: desc->C may exceed the master's Cin (c_master); pad lanes are 0. */
int mmdx_conv_pack_weight(int dtype, const mmdx_conv_desc* d, int c_master,
                          const float* w_kcrs, void* w_krsc, void* w_crsk, void* stream);
/* Every conv weight of a network in one launch.  items: DEVICE array of n_items, sorted by
 * first_block; item i owns blocks [first_block_i, first_block_{i+1}) (the last runs to
 * total_blocks), mmdx_conv_pack_blocks(K, C, R*S) of them.  Same packing as
 * mmdx_conv_pack_weight for unpadded weights: c_master must equal C (channel-padded weights
 * use mmdx_conv_pack_weight).  Items with RS = 1 and no crsk are plain [K][C] casts: the
 * transformer encoder stacks cast every layer's weights with one such launch (bf16 / fp16). */
typedef struct {
  const float* w;      /* fp32 KCRS master */
  void* krsc;          /* packed [K][R][S][C] or NULL */
  void* crsk;          /* packed [C][R][S][K] or NULL */
  int K, C, c_master, RS;
  long first_block;
} mmdx_pack_item;
long mmdx_conv_pack_blocks(int K, int C, int RS);
int mmdx_conv_pack_multi(int dtype, const mmdx_pack_item* items, int n_items, long total_blocks,
                         void* stream);
/* stat_part (optional, fp32 pairs [K][mmdx_conv_fwd_stat_blocks(d)], channel-major): per-channel
 * (mean, M2) of each mmdx_conv_fwd_stat_rows(d)-row block of the output (128 rows; the direct
 * pixel-pair stem kernel: one block of 2 output rows), computed from the fp32 accumulators in
 * the GEMM epilogue — the BatchNorm batch statistics without a separate pass over y
 * (replaces the BatchNorm2d reduction after backbone convs, TP:183 / torchvision). */
int mmdx_conv_fwd_stat_blocks(const mmdx_conv_desc* d);
int mmdx_conv_fwd_stat_rows(const mmdx_conv_desc* d);
int mmdx_conv_fwd(int dtype, const mmdx_conv_desc* d, const void* x, const void* w_krsc,
                  void* y, float* stat_part, void* stream);
/* The same with the statistics slab size the caller allocated stat_part for (stat_rows =
 * mmdx_conv_fwd_stat_rows(d) when the buffer was sized; a plan built once keeps its layout
 * whatever MMDX_STEM_DIRECT says later; a size the kernels cannot write is an error). */
int mmdx_conv_fwd_rows(int dtype, const mmdx_conv_desc* d, const void* x, const void* w_krsc,
                       void* y, float* stat_part, int stat_rows, void* stream);
/* Eval-mode conv + BatchNorm2d (running statistics) (+residual) (+ReLU) in one launch:
 * y = act(conv(x, w) * s + t + residual), s = gamma / sqrt(running_var + eps),
 * t = beta - running_mean * s, applied in the conv epilogue on the fp32 accumulators.
 * Replaces conv + bn_apply for the backbone in eval mode (TP:206 freeze_backbone, TP:1000
 * encoders in eval, IP:170 inference).  residual may be NULL. */
int mmdx_conv_fwd_bn_eval(int dtype, const mmdx_conv_desc* d, const void* x,
                          const void* w_krsc, void* y, const float* gamma, const float* beta,
                          const float* running_mean, const float* running_var, float eps,
                          const void* residual, int relu, void* stream);
/* dx = dgrad + beta * dx  (beta = 1 sums the residual-path gradient in the epilogue) */
int mmdx_conv_dgrad(int dtype, const mmdx_conv_desc* d, const void* dy,
                    const void* w_crsk, void* dx, float beta, void* stream);
/* dx = dgrad + beta * dx and, in the same epilogue, the backward statistics of the
 * BatchNorm whose output gradient the final dx is (its input bn_y, affine, saved mean/rstd):
 * stat_part [C][mmdx_conv_dgrad_stat_blocks()] (sum g, sum g*xhat) per 128-row tile, for
 * mmdx_bn_bwd.  The ReLU mask is bn_out > 0 for a residual unit (bn_out = its output
 * relu(bn(y) + res)), else recomputed from bn_y with the forward's scale/shift (bn_out NULL).
 * beta != 0 (accumulating a residual branch's gradient) needs a stride-1 conv.
 * stat_blocks == 0: the fusion does not apply to this conv. */
int mmdx_conv_dgrad_stat_blocks(int dtype, const mmdx_conv_desc* d);
int mmdx_conv_dgrad_bnstat(int dtype, const mmdx_conv_desc* d, const void* dy,
                           const void* w_crsk, void* dx, float beta, const void* bn_y,
                           const void* bn_out, const float* gamma, const float* bn_beta,
                           const float* save_mean, const float* save_rstd, int relu,
                           float* stat_part, void* stream);
/* stride-1 dgrad whose epilogue adds a masked tensor: dx = dgrad(dy) + (bit ? acc_src : 0),
 * the bit from a 1-bit ReLU mask written by mmdx_bn_fwd_ex ([rows][C / (16 / elem)] bytes).
 * An identity block's conv1 dgrad adds the gradient that reached the block output through
 * the residual unit's ReLU (its dout, masked) — mmdx_bn_bwd then writes no d_residual.
 * Equals mmdx_conv_dgrad with beta 1 onto that masked gradient, bit for bit. */
int mmdx_conv_dgrad_accmask(int dtype, const mmdx_conv_desc* d, const void* dy,
                            const void* w_crsk, void* dx, const void* acc_src,
                            const uint8_t* acc_mask, void* stream);
size_t mmdx_conv_wgrad_workspace_size(int dtype, const mmdx_conv_desc* d);
/* dw_kcrs (fp32, master layout, Cin = c_master) = dw_kcrs*beta + grad */
int mmdx_conv_wgrad(int dtype, const mmdx_conv_desc* d, int c_master, const void* x,
                    const void* dy, float* dw_kcrs, float beta, void* workspace,
                    size_t ws_bytes, void* stream);

/* ResNet stem (backbone.0, TP:183: 7x7 / stride 2 / pad 3 over the 3-channel image) as an
 * ordinary conv over PIXEL PAIRS (bf16 path): the NCHW fp32 batch of
 * image_transfom_into_tensor (TP:112-119) is written once, zero-bordered, as
 * [N][H+2p][(W+2p)/2][8] bf16 (two adjacent padded pixels x 4 channels per "pixel"); the
 * stem is then a stride (2,1), unpadded R x ceil(S/2) conv with 8 channels (K = 224 instead of
 * 392 for the channel-padded image, no border taps) run by mmdx_conv_fwd / mmdx_conv_wgrad
 * with the descriptor mmdx_stem_pair_desc returns.  Needs stride 2, C <= 4, even W + 2p.
 *   pack:  w_kcrs fp32 [K][C][R][S] -> w_packed [K][R][ceil(S/2)][8] bf16 (the pair conv's KRSC)
 *   grad:  dw_pair fp32 [K][8][R][ceil(S/2)] (mmdx_conv_wgrad of the pair conv, c_master 8)
 *          -> dw_kcrs (master layout) = beta * dw_kcrs + grad */
int mmdx_stem_pair_desc(int N, int C, int H, int W, int K, int R, int S, int stride, int pad,
                        mmdx_conv_desc* out);
int mmdx_stem_pair_input(const float* x_nchw, int N, int C, int H, int W, int pad, void* out,
                         void* stream);
int mmdx_stem_pair_pack_weight(const float* w_kcrs, int K, int C, int R, int S, void* w_packed,
                               void* stream);
int mmdx_stem_pair_grad(const float* dw_pair, int K, int C, int R, int S, float* dw_kcrs,
                        float beta, void* stream);

/* ---------------------------------------------------------------- batch norm (+res)(+ReLU)
 * x, y, residual: [rows, C] (NHWC flattened).  Train mode computes batch statistics
 * (biased var for normalisation, unbiased for running_var, momentum update as
 * nn.BatchNorm2d(eps, momentum)); eval mode uses running stats.
 * save_mean/save_rstd: [C] fp32, consumed by the backward.
 * Replaces: BatchNorm2d + ReLU (+ Bottleneck residual add) inside the resnet trunk
 * (train mode: unfreeze_backbone TP:223; eval: freeze_backbone TP:206, IP:170). */
size_t mmdx_bn_workspace_size(long rows, int C);
/* stat_part: optional precomputed per-block (mean, M2) pairs [C][stat_blocks] over
 * consecutive stat_rows-row blocks (e.g. from mmdx_conv_fwd's epilogue); NULL = reduce x. */
int mmdx_bn_fwd(int dtype, int train, const void* x, long rows, int C,
                const float* stat_part, int stat_blocks, long stat_rows,
                const float* gamma, const float* beta, float* running_mean,
                float* running_var, float momentum, float eps,
                float* save_mean, float* save_rstd,
                const void* residual, int relu, void* y,
                void* workspace, size_t ws_bytes, void* stream);
/* y == NULL (train): statistics only — save_mean/save_rstd and the running-stat update, no
 * apply pass (the consumer normalises on the fly, e.g. mmdx_maxpool_bn_fwd). */
/* mmdx_bn_fwd plus, when relu_mask != NULL (relu units): one byte per 16-B channel vector of
 * each row ([rows][C / (16 / sizeof(dtype))]), bit e set iff the stored y element e is > 0 —
 * the ReLU mask mmdx_bn_bwd_ex reads instead of y (1 bit per element instead of 16). */
int mmdx_bn_fwd_ex(int dtype, int train, const void* x, long rows, int C,
                   const float* stat_part, int stat_blocks, long stat_rows,
                   const float* gamma, const float* beta, float* running_mean,
                   float* running_var, float momentum, float eps,
                   float* save_mean, float* save_rstd,
                   const void* residual, int relu, void* y, uint8_t* relu_mask,
                   void* workspace, size_t ws_bytes, void* stream);
/* The two halves of the train forward above: the finalize of precomputed slabs (mean,
 * rstd, running stats, scale = gamma*rstd, shift = beta - mean*scale), and the apply pass
 * y = act(x*scale + shift (+ residual)) with the optional ReLU bit mask. */
int mmdx_bn_finalize(const float* stat_part, int stat_blocks, long stat_rows, long rows, int C,
                     const float* gamma, const float* beta, float* running_mean,
                     float* running_var, float momentum, float eps, float* save_mean,
                     float* save_rstd, float* scale, float* shift, void* stream);
int mmdx_bn_apply(int dtype, const void* x, const void* residual, long rows, int C,
                  const float* scale, const float* shift, int relu, void* y,
                  uint8_t* relu_mask, void* stream);
/* dy: grad w.r.t. y; y: forward output (ReLU mask source).  Writes dx, d_residual
 * (may be NULL), and dgamma/dbeta (fp32, accumulated with beta_acc). */
int mmdx_bn_bwd(int dtype, int train, const void* x, const void* y, const void* dy,
                long rows, int C, const float* gamma, const float* bn_beta,
                const float* save_mean, const float* save_rstd, int relu,
                const float* stat_part, int stat_blocks, void* dx,
                void* d_residual, float* dgamma, float* dbeta, float beta_acc,
                void* workspace, size_t ws_bytes, void* stream);
/* mmdx_bn_bwd with the ReLU mask taken from relu_mask (written by mmdx_bn_fwd_ex) when it is
 * not NULL — a residual unit's backward then reads 1 bit per element instead of its output;
 * results are identical to mmdx_bn_bwd with y. */
int mmdx_bn_bwd_ex(int dtype, int train, const void* x, const void* y, const void* dy,
                   long rows, int C, const float* gamma, const float* bn_beta,
                   const float* save_mean, const float* save_rstd, int relu,
                   const float* stat_part, int stat_blocks, void* dx,
                   void* d_residual, float* dgamma, float* dbeta, float beta_acc,
                   const uint8_t* relu_mask, void* workspace, size_t ws_bytes, void* stream);
/* BN backward (no ReLU, no residual: a downsample branch's BN) whose upstream gradient is
 * dy with a 1-bit ReLU mask applied on the fly (dy_mask from mmdx_bn_fwd_ex of the residual
 * unit whose identity path feeds it) — equals mmdx_bn_bwd on the materialised masked dy. */
int mmdx_bn_bwd_masked_dy(int dtype, int train, const void* x, const void* dy,
                          const uint8_t* dy_mask, long rows, int C, const float* gamma,
                          const float* bn_beta, const float* save_mean,
                          const float* save_rstd, void* dx, float* dgamma, float* dbeta,
                          float beta_acc, void* workspace, size_t ws_bytes, void* stream);
/* stat_part (optional, [C][stat_blocks] pairs (sum g, sum g*xhat)): the reduction already
 * made by mmdx_conv_dgrad_bnstat in the epilogue that produced dy — the BN backward then
 * skips its own pass over (dy, x).  ReLU units only (with y = the unit's output for a
 * residual unit, y == NULL otherwise). */
/* relu with y == NULL (a unit without residual): the ReLU mask is recomputed from x as
 * x*scale + shift > 0 with the forward's own scale/shift (gamma, bn_beta, save_mean,
 * save_rstd), so the post-activation tensor is not read. */

/* The stem's BN backward reading its upstream gradient straight from the 3x3 / stride-2
 * pool's output gradient dy_pooled [N][P][Q][C] and argmax (mmdx_maxpool_fwd /
 * mmdx_maxpool_bn_fwd): dL/d(pool input) is gathered on the fly (rounded to the compute dtype,
 * as mmdx_maxpool_bwd stores it), so the result equals mmdx_maxpool_bwd followed by
 * mmdx_bn_bwd (y == NULL, no residual) without materialising the [N][H][W][C] gradient.
 * x: the stem conv's raw output [N][H][W][C]. */
int mmdx_bn_bwd_pool(int dtype, int train, const void* x, const uint8_t* argmax,
                     const void* dy_pooled, int N, int H, int W, int C, int k, int s, int p,
                     int P, int Q, const float* gamma, const float* bn_beta,
                     const float* save_mean, const float* save_rstd, int relu, void* dx,
                     float* dgamma, float* dbeta, float beta_acc, void* workspace,
                     size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- launch plans
 * A plan is a host array of operations over caller-owned buffers, recorded once by the
 * host layer (the ResNet trunk forward or backward for one batch shape and parameter set)
 * and replayed with ONE call per step, so the per-step host cost is the launches alone.
 * Operand j of an op is o.p[j] itself when o.ext[j] < 0, else ext[o.ext[j]] + (intptr)o.p[j]
 * (per-call buffers: the image batch, the upstream gradient, the gradient arena).
 * Each op runs on streams[o.stream] (streams[0] = the caller's stream).  MMDX_OP_EVENT
 * records timing event events[o.i[0]] (skipped when events is NULL); MMDX_OP_SIGNAL records
 * the hipEvent_t o.p[0] on the op's stream and MMDX_OP_WAIT makes the op's stream wait on it
 * (cross-stream order inside a plan: e.g. weight gradients on a side stream).
 * Argument packing per op: see csrc/plan.cpp (each op forwards to the entry point of the
 * same name above/below with its i/l/f/p fields in signature order).
 * Replaces: the per-layer Python dispatch of ImageEncoderCNN's trunk (TP:279-289) and of
 * the BERT / ViT encoder layers (TP:360/470 AutoModel's BertLayer stack; vit_b_16). */
enum {
  MMDX_OP_EVENT = 1, MMDX_OP_NCHW2NHWC, MMDX_OP_CONV_PACK, MMDX_OP_CONV_FWD, MMDX_OP_BN_FWD,
  MMDX_OP_MAXPOOL_FWD, MMDX_OP_AVGPOOL_FWD, MMDX_OP_CAST, MMDX_OP_AVGPOOL_BWD,
  MMDX_OP_MAXPOOL_BWD, MMDX_OP_BN_BWD, MMDX_OP_CONV_WGRAD, MMDX_OP_CONV_DGRAD,
  MMDX_OP_SIGNAL, MMDX_OP_WAIT, MMDX_OP_CONV_DGRAD_BNSTAT, MMDX_OP_STEM_PAIR_INPUT,
  MMDX_OP_STEM_PAIR_PACK, MMDX_OP_STEM_PAIR_GRAD, MMDX_OP_CONV_PACK_MULTI,
  MMDX_OP_CONV_FWD_BNEVAL, MMDX_OP_MAXPOOL_BN_FWD, MMDX_OP_BN_BWD_POOL,
  MMDX_OP_CONV_DGRAD_ACCMASK, MMDX_OP_BN_BWD_MASKED_DY,
  /* transformer layer stacks (BERT / ViT encoders, one plan per stack and direction) */
  MMDX_OP_GEMM, MMDX_OP_ATTN_FWD, MMDX_OP_ATTN_BWD, MMDX_OP_LN_FWD, MMDX_OP_LN_BWD,
  MMDX_OP_GELU_BWD, MMDX_OP_BIAS_GRAD, MMDX_OP_ADD, MMDX_OP_DROPOUT_FWD, MMDX_OP_DROPOUT_BWD,
  MMDX_OP_AXPBY, MMDX_OP_ATTN_FWD_LSE, MMDX_OP_ATTN_BWD_LSE, MMDX_OP_LN_FWD_DROP,
  MMDX_OP_LN_BWD_DROP, MMDX_OP_GEMM_BIAS_GRAD,
  /* (42: the retired conv + fused BN finalize op, tools/lab/RETIRED.md) and the BN apply pass
   * (i: C, relu; l: rows; p: x, residual, scale, shift, y, relu_mask) */
  MMDX_OP_RETIRED_42, MMDX_OP_BN_APPLY
};
typedef struct {
  int op, dtype, stream;
  int i[8];
  long l[4];
  float f[4];
  const void* p[12];
  int ext[12];
  mmdx_conv_desc d;
} mmdx_plan_op;
int mmdx_plan_run(const mmdx_plan_op* ops, int n_ops, void* const* ext, void* const* events,
                  void* const* streams, int n_streams);
size_t mmdx_plan_op_size(void); /* sizeof(mmdx_plan_op): binding layout check */

/* ---------------------------------------------------------------- pooling
 * Replaces: resnet maxpool 3x3/2 (backbone[3]) and AdaptiveAvgPool2d(1) (backbone[8])
 * followed by flatten(1) (TP:281/288). */
/* argmax: uint8 window index (r*k+s) of the first maximum, as PyTorch CPU max_pool2d */
int mmdx_maxpool_fwd(int dtype, const void* x, int N, int H, int W, int C, int k, int s,
                     int p, void* y, uint8_t* argmax, int P, int Q, void* stream);
/* The stem's BN(+ReLU) fused into its 3x3 / stride-2 pool (train forward): x is the RAW stem
 * conv output; every tap is normalised with the batch statistics mmdx_bn_fwd saved (called
 * with y == NULL: statistics, running stats and save_mean/save_rstd only, no apply pass), as
 * scale = gamma*rstd, shift = beta - mean*gamma*rstd, ReLU'd and rounded to the compute dtype
 * before the compare — y and argmax are bit-identical to mmdx_bn_fwd's apply followed by
 * mmdx_maxpool_fwd, without writing or re-reading the post-activation tensor.
 * Replaces: backbone[1..3] (BatchNorm2d, ReLU, MaxPool2d) of the trunk, TP:183/279-281. */
int mmdx_maxpool_bn_fwd(int dtype, const void* x, int N, int H, int W, int C, int k, int s,
                        int p, const float* gamma, const float* beta, const float* save_mean,
                        const float* save_rstd, int relu, void* y, uint8_t* argmax, int P, int Q,
                        void* stream);
int mmdx_maxpool_bwd(int dtype, const uint8_t* argmax, const void* dy, int N, int H, int W,
                     int C, int k, int s, int p, int P, int Q, void* dx, void* stream);
int mmdx_avgpool_fwd(int dtype, const void* x, int N, int HW, int C, void* y, void* stream);
int mmdx_avgpool_bwd(int dtype, const void* dy, int N, int HW, int C, void* dx,
                     void* stream);

/* ---------------------------------------------------------------- layout / casts
 * NCHW fp32 image batch (output of image_transfom_into_tensor, TP:112-119) ->
 * NHWC compute dtype with channels zero-padded to c_pad. */
int mmdx_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, int c_pad,
                      void* y, void* stream);
int mmdx_cast(int dst_dtype, int src_dtype, const void* x, long n, void* y, void* stream);
/* out = a*x + b*y (fp32; y may be NULL) — bias folding (LSTM b_ih + b_hh), grad copies */
int mmdx_axpby(long n, float a, const float* x, float b, const float* y, float* out,
               void* stream);

/* ---------------------------------------------------------------- ViT-B/16 tower (C5)
 * torchvision vit_b_16 (build-defined backbone name):
 * patchify: x NCHW fp32 -> [N*(H/p)*(W/p)][C*p*p] rows in (c, ky, kx) order, so the
 *   Conv2d(C, D, p, stride p) patch embedding is one GEMM against its [D][C*p*p] weight;
 * vit_tokens: tokens[n][0] = class_token + pos[0], tokens[n][1+q] = emb[n][q] + pos[1+q];
 *   backward returns d emb (the class-token / pos gradients are column sums, bias_grad);
 * rows_copy: strided row copy (class-token rows in and out of the token matrix);
 * add: out = x + y in the compute dtype (residual gradient sums). */
int mmdx_patchify(int dtype, const float* x, int N, int C, int H, int W, int p, void* out,
                  void* stream);
int mmdx_vit_tokens_fwd(int dtype, const void* emb, const float* cls, const float* pos, int N,
                        int S, int D, void* tokens, void* stream);
int mmdx_vit_tokens_bwd(int dtype, const void* dtokens, int N, int S, int D, void* demb,
                        void* stream);
int mmdx_rows_copy(int dtype, const void* src, long src_ld, void* dst, long dst_ld, long rows,
                   int D, void* stream);
int mmdx_add(int dtype, long n, const void* x, const void* y, void* out, void* stream);

/* ---------------------------------------------------------------- image preprocessing
 * Batched GPU version of image_transfom_into_tensor (TP:112-119): torchvision
 * Resize(256, antialias=True) on a PIL image (= PIL ImagingResample, bilinear filter, two
 * fixed-point passes, horizontal first, 22-bit coefficients, uint8 clipped after each pass),
 * CenterCrop(224), ToTensor, gray->RGB repeat, Normalize(ImageNet).  Bit-exact with the CPU
 * transform.  pixels: the batch's decoded HWC uint8 images (JPEG decode stays on the host,
 * PIL, TP:146) packed back to back; descs/coef: per-image geometry and PIL coefficient
 * tables (host-computed, mmdx.preprocess); temp: >= sum of trows*out_w*c bytes;
 * out: [B][3][out_h][out_w] fp32. */
typedef struct {
  long src_off;         /* byte offset of the image's HWC pixels */
  long kh_off, kv_off;  /* int offsets into coef: per crop column / row {min, count, k[ksize]} */
  long temp_off;        /* byte offset of the image's [trows][out_w][c] intermediate */
  int w, h, c;          /* source width, height, channels (1 = L, 3 = RGB) */
  int left, top;        /* crop origin in the resized image */
  int need_h, need_v;   /* which PIL resample passes run */
  int ksize_h, ksize_v; /* coefficients per output column / row */
  int trow0, trows;     /* source rows the horizontal pass covers */
} mmdx_img_desc;
size_t mmdx_img_desc_size(void); /* sizeof(mmdx_img_desc): binding layout check */
int mmdx_image_preprocess(const uint8_t* pixels, const mmdx_img_desc* descs, int B,
                          const int* coef, int max_trows, int out_h, int out_w, uint8_t* temp,
                          float* out, void* stream);

/* ---------------------------------------------------------------- elementwise / norms
 * LayerNorm over the last dim D (fusion_mlp[3] TP:538, BERT LayerNorms);
 * optional residual added before the norm (BERT "Add & Norm"). */
int mmdx_layernorm_fwd(int dtype, const void* x, const void* residual, long rows, int D,
                       const float* gamma, const float* beta, float eps, void* y,
                       void* sum_out, float* save_mean, float* save_rstd, void* stream);
int mmdx_layernorm_bwd(int dtype, const void* xsum, const void* dy, long rows, int D,
                       const float* gamma, const float* save_mean, const float* save_rstd,
                       void* dx, float* dgamma, float* dbeta, float beta_acc,
                       void* workspace, size_t ws_bytes, void* stream);
size_t mmdx_layernorm_workspace_size(long rows, int D);
/* LayerNorm(dropout(x) + residual) in one pass (BertSelfOutput / BertOutput in train mode):
 * element e of x is kept with the keep bit mmdx_dropout_fwd would draw for it (seed,
 * *counter), scaled by 1/(1-p) and rounded to dtype as that kernel stores it, so the outputs
 * are bit-identical to mmdx_dropout_fwd + mmdx_layernorm_fwd with neither the dropped tensor
 * nor its mask written.  rng[0] (device uint64) receives the stream base for the backward;
 * counter (may be NULL) is incremented after the launch.
 * Replaces: BertSelfOutput.dropout + LayerNorm, BertOutput.dropout + LayerNorm (TP:360). */
int mmdx_layernorm_fwd_dropout(int dtype, const void* x, const void* residual, long rows,
                               int D, const float* gamma, const float* beta, float eps, float p,
                               uint64_t seed, uint64_t* counter, void* y, void* sum_out,
                               float* save_mean, float* save_rstd, uint64_t* rng, void* stream);
/* mmdx_layernorm_bwd with a residual branch's gradient added to dx before its one rounding:
 * dx = LN'(dy) + residual_grad (the pre-LN encoder block's "x + f(LN(x))" backward, vit_b_16);
 * residual_grad must not alias dx. */
int mmdx_layernorm_bwd_residual(int dtype, const void* xsum, const void* dy, long rows, int D,
                                const float* gamma, const float* save_mean,
                                const float* save_rstd, const void* residual_grad, void* dx,
                                float* dgamma, float* dbeta, float beta_acc, void* workspace,
                                size_t ws_bytes, void* stream);
/* mmdx_layernorm_bwd plus dx_drop = the dropout backward of dx with the keep bits of rng[0]
 * (bit-identical to mmdx_dropout_bwd on dx and the forward's mask). */
int mmdx_layernorm_bwd_dropout(int dtype, const void* xsum, const void* dy, long rows, int D,
                               const float* gamma, const float* save_mean,
                               const float* save_rstd, float p, const uint64_t* rng, void* dx,
                               void* dx_drop, float* dgamma, float* dbeta, float beta_acc,
                               void* workspace, size_t ws_bytes, void* stream);
/* GELU backward from the pre-activation: dx = dy * gelu'(pre) */
int mmdx_gelu_bwd(int dtype, const void* pre, const void* dy, long n, void* dx,
                  void* stream);
/* bias gradient: db[N] (+)= sum_m dy[m, N] */
int mmdx_bias_grad(int dtype, const void* dy, long M, int N, float* db, float beta_acc,
                   void* workspace, size_t ws_bytes, void* stream);
size_t mmdx_bias_grad_workspace_size(long M, int N);
/* dropout with a counter-based hash RNG: y = x * mask / (1-p); mask saved as uint8.
 * counter: optional device uint64.  When given, the RNG stream is (seed, offset + *counter
 * << 32) and *counter is incremented after the launch (stream-ordered), so the call can be
 * captured in a hipGraph and every replay draws a fresh mask (torch.nn.Dropout, TP:538). */
int mmdx_dropout_fwd(int dtype, const void* x, long n, float p, uint64_t seed,
                     uint64_t offset, uint64_t* counter, void* y, uint8_t* mask, void* stream);
int mmdx_dropout_bwd(int dtype, const void* dy, const uint8_t* mask, long n, float p,
                     void* dx, void* stream);

/* ---------------------------------------------------------------- loss / heads
 * BCEWithLogitsLoss (mean) (TP:843,1015,1049): loss[0] = mean over B*C;
 * dlogits = (sigmoid(z) - y) / (B*C) * dloss_scale. */
int mmdx_bce_logits_fwd(const float* logits, const float* target, int B, int C,
                        float* loss, void* stream);
int mmdx_bce_logits_bwd(const float* logits, const float* target, int B, int C,
                        const float* dloss, float* dlogits, void* stream);

/* ---------------------------------------------------------------- text towers
 * BERT embeddings: word[id] + pos[i] + type[tt] -> LayerNorm (transformers BertEmbeddings,
 * reached from TextEncoderTransformer.encode TP:470/473).  ids/tt int64 [B,L]. */
int mmdx_embed_ln_fwd(int dtype, const int64_t* ids, const int64_t* tt, int B, int L,
                      int D, const float* word, const float* pos, const float* type,
                      const float* gamma, const float* beta, float eps, void* y,
                      void* xsum, float* save_mean, float* save_rstd, void* stream);
/* scatter-add (+=) of dx (= grad of the pre-LN sum) into dense fp32 table grads;
 * rows with id == pad_id get no gradient (nn.Embedding padding_idx; -1 = none) */
int mmdx_embed_bwd(int dtype, const int64_t* ids, const int64_t* tt, int B, int L, int D,
                   const void* dsum, float* dword, float* dpos, float* dtype_tab,
                   int pad_id, void* stream);
/* masked mean pool (TP:452-459): out[b,:] = sum_l h[b,l,:]*m[b,l] / max(sum_l m, 1e-6) */
int mmdx_masked_mean_fwd(int dtype, const void* h, const int64_t* mask, int B, int L,
                         int D, void* out, void* stream);
int mmdx_masked_mean_bwd(int dtype, const void* dout, const int64_t* mask, int B, int L,
                         int D, void* dh, void* stream);
/* fused embedding gather + masked mean (build-defined C2 text tower):
 * out[b,:] = sum_l E[ids[b,l],:]*m[b,l] / max(sum_l m, 1e-6) */
int mmdx_embed_mean_fwd(int dtype, const int64_t* ids, const int64_t* mask, int B, int L,
                        int D, const float* table, void* out, void* stream);
int mmdx_embed_mean_bwd(int dtype, const int64_t* ids, const int64_t* mask, int B, int L,
                        int D, const void* dout, float* dtable, void* stream);
/* embedding gather (rows of an fp32 table -> compute dtype), for the BiLSTM tower */
int mmdx_embed_gather(int dtype, const int64_t* ids, long n, int D, const float* table,
                      void* out, void* stream);
int mmdx_embed_scatter(int dtype, const int64_t* ids, long n, int D, const void* dout,
                       float* dtable, void* stream);

/* Multi-head self-attention core, head dim 64, L <= 256, additive key mask
 * (BertSelfAttention: softmax(QK^T*scale + (1-mask)*(-huge)) V; mask may be NULL = ViT).
 * qkv: [B, L, 3, H, 64] (fused projection output); out: [B, L, H, 64];
 * probs saved for backward: [B, H, L, L] fp32 (NULL in inference).
 * p_drop > 0 (training, BertSelfAttention's dropout on attention_probs): O = (P*keep/(1-p)) V
 * with keep drawn from a counter-based hash of (seed, *counter, b, h, q, key); the saved
 * probabilities carry keep in their sign bit (dropped: -P), so the backward needs neither
 * RNG nor a mask.  counter (device uint64, may be NULL) is incremented after the launch.
 * dqkv: [B, L, 3, H, 64]; workspace holds dS ([B,H,L,roundup32(L)] compute dtype). */
int mmdx_attention_fwd(int dtype, const void* qkv, const int64_t* mask, int B, int L,
                       int H, float scale, float p_drop, uint64_t seed, uint64_t* counter,
                       void* out, float* probs, void* stream);
/* As mmdx_attention_fwd, plus an additive fp32 score bias [H][L][L] shared by the batch
 * (T5's relative position bias; NULL = none) and a causal mask (key > query masked). */
int mmdx_attention_fwd_ex(int dtype, const void* qkv, const int64_t* mask, const float* bias,
                          int causal, int B, int L, int H, float scale, float p_drop,
                          uint64_t seed, uint64_t* counter, void* out, float* probs,
                          void* stream);
/* The backward leaves dS (the score gradient = the bias gradient) in the workspace as
 * [B][H][L][roundup32(L)] compute dtype, for mmdx_t5_position_bias_bwd. */
size_t mmdx_attention_workspace_size(int dtype, int B, int L, int H);
int mmdx_attention_bwd(int dtype, const void* qkv, const float* probs, const void* dout,
                       const int64_t* mask, int B, int L, int H, float scale, float p_drop,
                       void* dqkv, void* workspace, size_t ws_bytes, void* stream);
/* Flash-style variant (16-bit dtypes, no score bias / causal mask): the forward saves the
 * row log-sum-exp lse [B, H, L] fp32 instead of P, and rng[0] (device uint64) receives the
 * dropout stream's base (seed and *counter as the launch read them).  The backward
 * recomputes P from Q, K and lse, the keep bits from the same hash, and the softmax row term
 * rowsum(P o dP) as dO . out (out = the forward's output, which the attention output
 * projection keeps anyway), so no [B, H, L, L] tensor is written or read.  The workspace
 * holds that row term ([B, H, L] fp32).  Same arguments and results otherwise.
 * Replaces: BertSelfAttention / torchvision MultiheadAttention as above (TP:360, vit_b_16). */
int mmdx_attention_fwd_lse(int dtype, const void* qkv, const int64_t* mask, int B, int L,
                           int H, float scale, float p_drop, uint64_t seed, uint64_t* counter,
                           void* out, float* lse, uint64_t* rng, void* stream);
size_t mmdx_attention_lse_workspace_size(int dtype, int B, int L, int H);
int mmdx_attention_bwd_lse(int dtype, const void* qkv, const void* out, const float* lse,
                           const uint64_t* rng, const void* dout, const int64_t* mask, int B,
                           int L, int H, float scale, float p_drop, void* dqkv,
                           void* workspace, size_t ws_bytes, void* stream);

/* LSTM recurrence for one layer, both directions (build-defined C3/C4 tower).
 * xg: [B, L, 2, H, 4] precomputed input gates (x W_ih^T + b_ih + b_hh), the four gates
 *     (i,f,g,o) of a unit adjacent;
 * w_hh: [2][4H][H] compute dtype; h_out: [B, L, 2H]; saved c: [2, L, B, H] fp32,
 * gates: [2, L, B, H, 4] fp32 post-activation, the four gates of a unit adjacent (for
 * backward). */
/* Workspace for the cooperative bf16 forward (H = 256, B <= 256): h exchange + counters.
 * 0 when that path does not apply (then ws may be NULL and the batch-partitioned kernel
 * runs).
 * status: DEVICE int, caller-owned, zero-initialised and STICKY: the cooperative kernel sets
 * it to 1 when a peer workgroup never arrives within spin_limit polls (<= 0: the default,
 * ~2 s) — every workgroup then leaves and the outputs are invalid.  The kernel never clears
 * it; the caller copies it to the host at a sync point and raises (bilstm.py).  A non-zero
 * status on entry makes the kernel leave at its first wait.  debug_flags bit 0 (tests
 * only): workgroup 0 of direction 0 never signals, forcing the timeout path; bit 1 (lab
 * probe, tools/lab/lstm_probe.py): per-step phase timestamps after the workspace (the
 * caller passes [groups][2][8][L][8] u64 more).
 * Returns -22 if the device cannot hold the cooperative grid resident. */
size_t mmdx_lstm_fwd_workspace_size(int dtype, int B, int L, int H);
int mmdx_lstm_fwd(int dtype, const void* xg, const void* w_hh, int B, int L, int H,
                  void* h_out, float* c_save, float* gates_save, void* workspace,
                  size_t ws_bytes, int* status, long spin_limit, int debug_flags,
                  void* stream);
size_t mmdx_lstm_workspace_size(int dtype, int B, int L, int H);
/* Backward.  status (may be NULL): the forward's device status word; with it, bf16, H = 256
 * and B <= 512 run the cooperative recurrence (4 workgroups per 16-row block and direction
 * exchanging dG slices, W_hh^T held in registers), whose bounded wait sets *status = 2 when
 * a peer never arrives within spin_limit polls (<= 0: the default).  NULL: the
 * batch-partitioned kernel.  Both use the same bf16 dG operand, packed fragments and k order;
 * their fp32 cell math may contract a multiply-add differently, and the recurrence carries
 * such a difference on, so the outputs agree to one bf16 ulp of the tensor's scale (most
 * elements exactly; tests/test_text_gpu.py).  debug_flags bit 0 (tests only): workgroup 0 of
 * direction 0 of the cooperative kernel never signals, so the peers' waits time out. */
int mmdx_lstm_bwd(int dtype, const void* w_hh, const void* h_out, const float* c_save,
                  const float* gates_save, const void* dh_out, int B, int L, int H,
                  void* dxg, float* dw_hh, void* workspace, size_t ws_bytes, int* status,
                  long spin_limit, int debug_flags, void* stream);

/* ---------------------------------------------------------------- T5 report head
 * (TP:545-618 cond_proj + T5ForConditionalGeneration, TP:983-991 /
 * TP:1049-1053 teacher-forced CE, IP:190-196 beam generate).  transformers' T5 arithmetic:
 * T5LayerNorm (RMSNorm, no mean / bias), unscaled self-attention with a relative-position
 * bias and a causal mask (mmdx_attention_fwd_ex), cross-attention over the K condition
 * tokens, ReLU FFN, tied lm_head on d_model^-0.5-scaled states, CE with ignore_index -100.
 * rmsnorm: y = w * x * rsqrt(mean(x^2) + eps); save_rstd [rows] fp32.
 * rmsnorm_bwd: dx = (grad) + beta * dx (beta = 1 adds onto a residual gradient);
 * dw (+)= dw_beta * dw + sum_rows dy * x * rstd (dw may be NULL). */
int mmdx_rmsnorm_fwd(int dtype, const void* x, long rows, int D, const float* w, float eps,
                     void* y, float* save_rstd, void* stream);
size_t mmdx_rmsnorm_workspace_size(long rows, int D);
int mmdx_rmsnorm_bwd(int dtype, const void* x, const void* dy, long rows, int D,
                     const float* w, const float* save_rstd, void* dx, float beta, float* dw,
                     float dw_beta, void* workspace, size_t ws_bytes, void* stream);
/* bias[h][q][k] = table[bucket(q - k)][h], table [num_buckets][H] (relative_attention_bias
 * .weight), causal (decoder) buckets of T5Attention._relative_position_bucket. */
int mmdx_t5_position_bias(const float* table, int H, int L, int num_buckets, int max_distance,
                          float* bias, void* stream);
/* dtable (+)= bucketed sum over batch and cells of dscores [B][H][L][ld] (compute dtype). */
int mmdx_t5_position_bias_bwd(int dtype, const void* dscores, int B, int H, int L, int ld,
                              int num_buckets, int max_distance, float* dtable, float beta,
                              void* stream);
/* Cross-attention over Lk <= 16 keys (the K condition tokens), head dim 64, no mask:
 * q rows [B][Lq] of ldq elements (head h at h*64); kv [B][Lk][2][H][64] (k then v);
 * out [B][Lq][H][64]; probs [B][H][Lq][Lk] fp32 (dropout keep bit in the sign, as
 * mmdx_attention_fwd).  dq rows of lddq elements; dkv like kv. */
int mmdx_xattn_fwd(int dtype, const void* q, long ldq, const void* kv, int B, int Lq, int Lk,
                   int H, float scale, float p_drop, uint64_t seed, uint64_t* counter,
                   void* out, float* probs, void* stream);
size_t mmdx_xattn_workspace_size(int B, int Lq, int Lk, int H);
int mmdx_xattn_bwd(int dtype, const void* q, long ldq, const void* kv, const float* probs,
                   const void* dout, int B, int Lq, int Lk, int H, float scale, float p_drop,
                   void* dq, long lddq, void* dkv, void* workspace, size_t ws_bytes,
                   void* stream);
/* CrossEntropyLoss(ignore_index=-100) mean over the rows whose target is in [0, V):
 * loss, count (device scalars).  The workspace keeps per-row log-sum-exp for the backward:
 * dlogits = (softmax - onehot) * dloss / count (dloss device scalar or NULL = 1). */
size_t mmdx_cross_entropy_workspace_size(long rows);
int mmdx_cross_entropy_fwd(const float* logits, const int64_t* targets, long rows, long V,
                           float* loss, float* count, void* workspace, size_t ws_bytes,
                           void* stream);
int mmdx_cross_entropy_bwd(int dtype, const float* logits, const int64_t* targets, long rows,
                           long V, const float* dloss, const float* count,
                           const void* workspace, void* dlogits, void* stream);
/* row-wise log_softmax (beam search scores) */
int mmdx_log_softmax(const float* logits, long rows, long V, float* out, void* stream);
/* dx = dy * (y > 0) (T5 DenseReluDense backward from the ReLU output) */
int mmdx_relu_bwd(int dtype, const void* y, const void* dy, long n, void* dx, void* stream);
/* One incremental decoder step of T5's causal self-attention over a KV cache (beam search of
 * report_model.generate, IP:190-196 / TP:613-618): qkv [R][3*H*64] of position `pos`;
 * caches [R][Lmax][H*64]; key j of row r is read from cache row slots[r*Lmax + j] (the beam's
 * ancestry, so reordering beams moves no cache data); bias [H][Lmax][Lmax] fp32 relative-
 * position bias (mmdx_t5_position_bias); out [R][H*64].  The step's K/V are appended at
 * (row r, pos).  Lmax <= 512. */
int mmdx_t5_decode_attn(int dtype, const void* qkv, int R, int H, int pos, int Lmax,
                        void* k_cache, void* v_cache, const int* slots, const float* bias,
                        void* out, void* stream);
/* Beam-search candidate step (GenerationMixin._beam_search's topk, IP:190 num_beams): per
 * batch row b, the k (<= 16) largest log_probs[b*nb + i][v] + run_scores[b*nb + i] over
 * (i, v), ordered by value desc then flat index i*V + v asc; out_idx = that flat index.
 * First writes -inf into log_probs at the n_ban (row, token) int pairs of ban_pairs
 * (no_repeat_ngram_size) and, when eos_ban >= 0, at column eos_ban (min_new_tokens). */
int mmdx_beam_topk(float* log_probs, int B, int nb, long V, const float* run_scores,
                   const int* ban_pairs, int n_ban, int eos_ban, int k, float* out_val,
                   long* out_idx, void* stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.AdamW (decoupled weight decay) over every tensor of every param group in
 * one launch (build_optimizer groups TP:238-269, TP:408-432; fusion optimiser
 * TP:1018-1023).  `table` is a DEVICE array of chunk descriptors: each parameter tensor is
 * split into chunks (host side, <= 64K elements) and each descriptor carries the chunk's
 * p/g/m/v pointers, its length n and its group's lr/wd; one workgroup per chunk.
 * step_dev (device fp32) is incremented by the call, so the update replays inside a
 * graph.  grad_scale (device scalar or NULL) multiplies every gradient: the clip
 * coefficient of clip_grad_norm_ (TP:1058). */
typedef struct {
  float* p;
  const float* g;
  float* m;
  float* v;
  long n;
  long off;   /* informational: element offset of the chunk in its tensor */
  float lr;
  float wd;
} mmdx_adamw_tensor;
int mmdx_adamw_multi(int nchunks, const mmdx_adamw_tensor* table, float beta1, float beta2,
                     float eps, float* step_dev, const float* grad_scale, void* stream);
/* global L2 norm of the .g fields of `table`; scale[0] = min(1, max_norm/(norm+1e-6))
 * (torch.nn.utils.clip_grad_norm_); max_norm <= 0 gives scale 1. */
size_t mmdx_grad_norm_workspace_size(int nchunks);
int mmdx_grad_norm(int nchunks, const mmdx_adamw_tensor* table, float max_norm, float* norm,
                   float* scale, void* workspace, size_t ws_bytes, void* stream);
/* in-place g *= scale[0] over the .g fields (the mul_ of clip_grad_norm_) */
int mmdx_scale_grads(int nchunks, const mmdx_adamw_tensor* table, const float* scale,
                     void* stream);
/* Refresh the .g column of a device chunk table in stream order, without a host->device
 * copy (the optimizer's gradient buffers move between steps): row r, whose tensor index is
 * row_tensor[r] (a DEVICE int array built with the table), gets
 * g = grads[row_tensor[r]] + off.  `grads` is a HOST array of n_tensors device pointers;
 * they travel as kernel arguments (256 per launch).  A small hipMemcpyAsync from pinned
 * memory made the issuing host thread wait for the stream on this runtime. */
int mmdx_adamw_patch_grads(int nchunks, mmdx_adamw_tensor* table, const int* row_tensor,
                           int n_tensors, const float* const* grads, void* stream);

/* Mixed-precision loss scaling: torch.cuda.amp.GradScaler as the fusion loop drives it
 * (TP:1025-1026 GradScaler(enabled=use_amp), TP:1056 scaler.scale(loss).backward(), TP:1058
 * clip_grad_norm_, TP:1060-1061 scaler.step / scaler.update).
 * mmdx_grad_norm_amp: as mmdx_grad_norm over gradients that hold loss_scale[0] * g;
 * found_inf[0] = 1 if any gradient is inf/NaN; scale[0] = clip coefficient / loss_scale[0],
 * the clip coefficient taken on the unscaled norm (unscale_first != 0: scaler.unscale_ before
 * the clip) or on the scaled one (0: the reference's order, clip then scaler.step).
 * mmdx_adamw_multi_amp: mmdx_adamw_multi that skips the whole step (no update, no step
 * count) when found_inf[0] != 0 (scaler.step's skip).
 * mmdx_amp_update_scale: scaler.update() (torch._amp_update_scale_): overflow -> scale *=
 * backoff_factor, tracker = 0; else every growth_interval clean steps scale *= growth_factor.
 * mmdx_mul_dev_scalar: out = x * s[0], fp32 (scaler.scale(loss) and its backward). */
int mmdx_grad_norm_amp(int nchunks, const mmdx_adamw_tensor* table, float max_norm,
                       const float* loss_scale, int unscale_first, float* norm, float* scale,
                       float* found_inf, void* workspace, size_t ws_bytes, void* stream);
int mmdx_adamw_multi_amp(int nchunks, const mmdx_adamw_tensor* table, float beta1, float beta2,
                         float eps, float* step_dev, const float* grad_scale,
                         const float* found_inf, void* stream);
int mmdx_amp_update_scale(float* scale, int* growth_tracker, const float* found_inf,
                          float growth_factor, float backoff_factor, int growth_interval,
                          void* stream);
int mmdx_mul_dev_scalar(const float* x, long n, const float* s, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MMDX_H_ */
