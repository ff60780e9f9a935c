// Launch plans: a host-side list of mmdx operations over caller-owned buffers, recorded
// once by the host layer (the ResNet trunk's forward or backward for one batch shape and
// parameter set) and replayed by ONE call per step.  The per-step host cost becomes the
// HIP launches themselves instead of ~60 us of Python per conv+BN unit; the 53-unit
// ResNet-50 trunk forward is one call, its backward another (SURVEY §3.3 train step).
#include <hip/hip_runtime.h>

#include "../../include/mmdx.h"

extern "C" void mmdx_set_error(const char* fmt, ...);

namespace {

// Resolve operand j of an op: absolute pointer, or byte offset into external base ext[j].
inline void* P(const mmdx_plan_op& o, int j, void* const* ext) {
  const int e = o.ext[j];
  if (e < 0) return (void*)o.p[j];
  return (char*)ext[e] + (intptr_t)o.p[j];
}

int hip_rc(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  mmdx_set_error("plan: %s: %s", what, hipGetErrorString(e));
  return -(int)e;
}

int run_one(const mmdx_plan_op& o, void* const* ext, void* const* events, void* s) {
  switch (o.op) {
    case MMDX_OP_SIGNAL:
      return hip_rc(hipEventRecord((hipEvent_t)o.p[0], (hipStream_t)s), "hipEventRecord");
    case MMDX_OP_WAIT:
      return hip_rc(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)o.p[0], 0),
                    "hipStreamWaitEvent");
    case MMDX_OP_EVENT:
      return events ? hip_rc(hipEventRecord((hipEvent_t)events[o.i[0]], (hipStream_t)s),
                             "hipEventRecord")
                    : 0;
    case MMDX_OP_NCHW2NHWC:
      return mmdx_nchw_to_nhwc(o.dtype, (const float*)P(o, 0, ext), o.i[0], o.i[1], o.i[2],
                               o.i[3], o.i[4], P(o, 1, ext), s);
    case MMDX_OP_CONV_PACK:
      return mmdx_conv_pack_weight(o.dtype, &o.d, o.i[0], (const float*)P(o, 0, ext),
                                   P(o, 1, ext), P(o, 2, ext), s);
    case MMDX_OP_CONV_FWD:  // i: rows per statistics slab (0: mmdx_conv_fwd's default)
      if (o.i[0] > 0)
        return mmdx_conv_fwd_rows(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext),
                                  (float*)P(o, 3, ext), o.i[0], s);
      return mmdx_conv_fwd(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext),
                           (float*)P(o, 3, ext), s);
    case MMDX_OP_CONV_FWD_BNEVAL:
      // i: relu; f: eps; p: x, w, y, gamma, beta, running_mean, running_var, residual
      return mmdx_conv_fwd_bn_eval(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext),
                                   (const float*)P(o, 3, ext), (const float*)P(o, 4, ext),
                                   (const float*)P(o, 5, ext), (const float*)P(o, 6, ext),
                                   o.f[0], P(o, 7, ext), o.i[0], s);
    case MMDX_OP_BN_FWD:
      // i: train, C, stat_blocks, relu; l: rows, stat_rows, ws_bytes; f: momentum, eps
      // p[11]: optional ReLU bit mask (mmdx_bn_fwd_ex)
      return mmdx_bn_fwd_ex(o.dtype, o.i[0], P(o, 0, ext), o.l[0], o.i[1],
                            (const float*)P(o, 1, ext), o.i[2], o.l[1],
                            (const float*)P(o, 2, ext), (const float*)P(o, 3, ext),
                            (float*)P(o, 4, ext), (float*)P(o, 5, ext), o.f[0], o.f[1],
                            (float*)P(o, 6, ext), (float*)P(o, 7, ext), P(o, 8, ext), o.i[3],
                            P(o, 9, ext), (uint8_t*)P(o, 11, ext), P(o, 10, ext),
                            (size_t)o.l[2], s);
    case MMDX_OP_MAXPOOL_FWD:
      // i: N, H, W, C, k, s, p, P ; l: Q
      return mmdx_maxpool_fwd(o.dtype, P(o, 0, ext), o.i[0], o.i[1], o.i[2], o.i[3], o.i[4],
                              o.i[5], o.i[6], P(o, 1, ext), (uint8_t*)P(o, 2, ext), o.i[7],
                              (int)o.l[0], s);
    case MMDX_OP_MAXPOOL_BN_FWD:
      // i: N, H, W, C, k, s, p, P ; l: Q, relu ; p: x, y, argmax, gamma, beta, mean, rstd
      return mmdx_maxpool_bn_fwd(o.dtype, P(o, 0, ext), o.i[0], o.i[1], o.i[2], o.i[3], o.i[4],
                                 o.i[5], o.i[6], (const float*)P(o, 3, ext),
                                 (const float*)P(o, 4, ext), (const float*)P(o, 5, ext),
                                 (const float*)P(o, 6, ext), (int)o.l[1], P(o, 1, ext),
                                 (uint8_t*)P(o, 2, ext), o.i[7], (int)o.l[0], s);
    case MMDX_OP_BN_BWD_POOL:
      // i: train, N, H, W, C, relu, P, Q ; l: ws_bytes, k, s, p ; f: beta_acc
      // p: x, argmax, dy_pooled, gamma, beta, mean, rstd, dx, dgamma, dbeta, ws
      return mmdx_bn_bwd_pool(o.dtype, o.i[0], P(o, 0, ext), (const uint8_t*)P(o, 1, ext),
                              P(o, 2, ext), o.i[1], o.i[2], o.i[3], o.i[4], (int)o.l[1],
                              (int)o.l[2], (int)o.l[3], o.i[6], o.i[7],
                              (const float*)P(o, 3, ext), (const float*)P(o, 4, ext),
                              (const float*)P(o, 5, ext), (const float*)P(o, 6, ext), o.i[5],
                              P(o, 7, ext), (float*)P(o, 8, ext), (float*)P(o, 9, ext), o.f[0],
                              P(o, 10, ext), (size_t)o.l[0], s);
    case MMDX_OP_AVGPOOL_FWD:
      return mmdx_avgpool_fwd(o.dtype, P(o, 0, ext), o.i[0], o.i[1], o.i[2], P(o, 1, ext), s);
    case MMDX_OP_CAST:
      return mmdx_cast(o.dtype, o.i[0], P(o, 0, ext), o.l[0], P(o, 1, ext), s);
    case MMDX_OP_AVGPOOL_BWD:
      return mmdx_avgpool_bwd(o.dtype, P(o, 0, ext), o.i[0], o.i[1], o.i[2], P(o, 1, ext), s);
    case MMDX_OP_MAXPOOL_BWD:
      return mmdx_maxpool_bwd(o.dtype, (const uint8_t*)P(o, 0, ext), P(o, 1, ext), o.i[0],
                              o.i[1], o.i[2], o.i[3], o.i[4], o.i[5], o.i[6], o.i[7],
                              (int)o.l[0], P(o, 2, ext), s);
    case MMDX_OP_BN_BWD:
      // i: train, C, relu, stat_blocks; l: rows, ws_bytes; f: beta_acc;
      // p: x, y, dy, gamma, beta, mean, rstd, dx, dres, dgamma, dbeta, ws; stat_part in l[2],
      // the optional ReLU bit mask (absolute pointer) in l[3]
      return mmdx_bn_bwd_ex(o.dtype, o.i[0], P(o, 0, ext), P(o, 1, ext), P(o, 2, ext), o.l[0],
                            o.i[1], (const float*)P(o, 3, ext), (const float*)P(o, 4, ext),
                            (const float*)P(o, 5, ext), (const float*)P(o, 6, ext), o.i[2],
                            (const float*)o.l[2], o.i[3], P(o, 7, ext), P(o, 8, ext),
                            (float*)P(o, 9, ext), (float*)P(o, 10, ext), o.f[0],
                            (const uint8_t*)o.l[3], P(o, 11, ext), (size_t)o.l[1], s);
    case MMDX_OP_BN_BWD_MASKED_DY:
      // i: train, C; l: rows, ws_bytes; f: beta_acc
      // p: x, dy, dy_mask, gamma, beta, mean, rstd, dx, dgamma, dbeta, ws
      return mmdx_bn_bwd_masked_dy(o.dtype, o.i[0], P(o, 0, ext), P(o, 1, ext),
                                   (const uint8_t*)P(o, 2, ext), o.l[0], o.i[1],
                                   (const float*)P(o, 3, ext), (const float*)P(o, 4, ext),
                                   (const float*)P(o, 5, ext), (const float*)P(o, 6, ext),
                                   P(o, 7, ext), (float*)P(o, 8, ext), (float*)P(o, 9, ext),
                                   o.f[0], P(o, 10, ext), (size_t)o.l[1], s);
    case MMDX_OP_CONV_DGRAD_ACCMASK:
      // p: dy, w_crsk, dx, acc_src, acc_mask
      return mmdx_conv_dgrad_accmask(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext),
                                     P(o, 3, ext), (const uint8_t*)P(o, 4, ext), s);
    case MMDX_OP_CONV_DGRAD_BNSTAT:
      // i: relu; f: beta; p: dy, w_crsk, dx, bn_y, gamma, beta, mean, rstd, stat_part, bn_out
      return mmdx_conv_dgrad_bnstat(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext),
                                    o.f[0], P(o, 3, ext), P(o, 9, ext),
                                    (const float*)P(o, 4, ext), (const float*)P(o, 5, ext),
                                    (const float*)P(o, 6, ext), (const float*)P(o, 7, ext),
                                    o.i[0], (float*)P(o, 8, ext), s);
    case MMDX_OP_CONV_WGRAD:
      // i: c_master; l: ws_bytes; f: beta
      return mmdx_conv_wgrad(o.dtype, &o.d, o.i[0], P(o, 0, ext), P(o, 1, ext),
                             (float*)P(o, 2, ext), o.f[0], P(o, 3, ext), (size_t)o.l[0], s);
    case MMDX_OP_CONV_DGRAD:
      return mmdx_conv_dgrad(o.dtype, &o.d, P(o, 0, ext), P(o, 1, ext), P(o, 2, ext), o.f[0],
                             s);
    case MMDX_OP_STEM_PAIR_INPUT:
      // i: N, C, H, W, pad; p: x_nchw, out
      return mmdx_stem_pair_input((const float*)P(o, 0, ext), o.i[0], o.i[1], o.i[2], o.i[3],
                                  o.i[4], P(o, 1, ext), s);
    case MMDX_OP_STEM_PAIR_PACK:
      // i: K, C, R, S; p: w_kcrs, w_packed
      return mmdx_stem_pair_pack_weight((const float*)P(o, 0, ext), o.i[0], o.i[1], o.i[2],
                                        o.i[3], P(o, 1, ext), s);
    case MMDX_OP_STEM_PAIR_GRAD:
      // i: K, C, R, S; f: beta; p: dw_pair, dw_kcrs
      return mmdx_stem_pair_grad((const float*)P(o, 0, ext), o.i[0], o.i[1], o.i[2], o.i[3],
                                 (float*)P(o, 1, ext), o.f[0], s);
    case MMDX_OP_CONV_PACK_MULTI:
      // i: n_items; l: total_blocks; p: item table (device)
      return mmdx_conv_pack_multi(o.dtype, (const mmdx_pack_item*)P(o, 0, ext), o.i[0], o.l[0],
                                  s);
    case MMDX_OP_GEMM:
      // i: M, N, K, a_kmajor, b_kmajor, c_dtype, act; l: lda, ldb, ldc, ws_bytes;
      // f: alpha, beta; p: A, B, C, bias, addend, preact, ws
      // (p[7]: optional residual, mmdx_gemm_res)
      if (P(o, 7, ext))
        return mmdx_gemm_res(o.dtype, o.i[0], o.i[1], o.i[2], P(o, 0, ext), o.l[0], o.i[3],
                             P(o, 1, ext), o.l[1], o.i[4], P(o, 2, ext), o.l[2], o.i[5],
                             (const float*)P(o, 3, ext), (const float*)P(o, 4, ext), o.i[6],
                             o.f[0], o.f[1], P(o, 5, ext), P(o, 7, ext), P(o, 6, ext),
                             (size_t)o.l[3], s);
      return mmdx_gemm(o.dtype, o.i[0], o.i[1], o.i[2], P(o, 0, ext), o.l[0], o.i[3],
                       P(o, 1, ext), o.l[1], o.i[4], P(o, 2, ext), o.l[2], o.i[5],
                       (const float*)P(o, 3, ext), (const float*)P(o, 4, ext), o.i[6], o.f[0],
                       o.f[1], P(o, 5, ext), P(o, 6, ext), (size_t)o.l[3], s);
    case MMDX_OP_GEMM_BIAS_GRAD:
      // i: M, N, K, c_dtype; l: lda, ldb, ldc, ws_bytes; p: A, B, C, db, ws
      return mmdx_gemm_bias_grad(o.dtype, o.i[0], o.i[1], o.i[2], P(o, 0, ext), o.l[0],
                                 P(o, 1, ext), o.l[1], P(o, 2, ext), o.l[2], o.i[3],
                                 (float*)P(o, 3, ext), P(o, 4, ext), (size_t)o.l[3], s);
    case MMDX_OP_ATTN_FWD:
      // i: B, L, H; f: scale, p_drop; l: seed; p: qkv, mask, counter, out, probs
      return mmdx_attention_fwd(o.dtype, P(o, 0, ext), (const int64_t*)P(o, 1, ext), o.i[0],
                                o.i[1], o.i[2], o.f[0], o.f[1], (uint64_t)o.l[0],
                                (uint64_t*)P(o, 2, ext), P(o, 3, ext), (float*)P(o, 4, ext), s);
    case MMDX_OP_ATTN_BWD:
      // i: B, L, H; f: scale, p_drop; l: ws_bytes; p: qkv, probs, dout, mask, dqkv, ws
      return mmdx_attention_bwd(o.dtype, P(o, 0, ext), (const float*)P(o, 1, ext), P(o, 2, ext),
                                (const int64_t*)P(o, 3, ext), o.i[0], o.i[1], o.i[2], o.f[0],
                                o.f[1], P(o, 4, ext), P(o, 5, ext), (size_t)o.l[0], s);
    case MMDX_OP_ATTN_FWD_LSE:
      // i: B, L, H; f: scale, p_drop; l: seed; p: qkv, mask, counter, out, lse, rng
      return mmdx_attention_fwd_lse(o.dtype, P(o, 0, ext), (const int64_t*)P(o, 1, ext), o.i[0],
                                    o.i[1], o.i[2], o.f[0], o.f[1], (uint64_t)o.l[0],
                                    (uint64_t*)P(o, 2, ext), P(o, 3, ext), (float*)P(o, 4, ext),
                                    (uint64_t*)P(o, 5, ext), s);
    case MMDX_OP_ATTN_BWD_LSE:
      // i: B, L, H; f: scale, p_drop; l: ws_bytes; p: qkv, out, lse, rng, dout, mask, dqkv, ws
      return mmdx_attention_bwd_lse(o.dtype, P(o, 0, ext), P(o, 1, ext), (const float*)P(o, 2, ext),
                                    (const uint64_t*)P(o, 3, ext), P(o, 4, ext),
                                    (const int64_t*)P(o, 5, ext), o.i[0], o.i[1], o.i[2], o.f[0],
                                    o.f[1], P(o, 6, ext), P(o, 7, ext), (size_t)o.l[0], s);
    case MMDX_OP_LN_FWD:
      // i: D; l: rows; f: eps; p: x, residual, gamma, beta, y, sum_out, mean, rstd
      return mmdx_layernorm_fwd(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                                (const float*)P(o, 2, ext), (const float*)P(o, 3, ext), o.f[0],
                                P(o, 4, ext), P(o, 5, ext), (float*)P(o, 6, ext),
                                (float*)P(o, 7, ext), s);
    case MMDX_OP_LN_BWD:
      // i: D; l: rows, ws_bytes; f: beta_acc; p: xsum, dy, gamma, mean, rstd, dx, dgamma,
      // dbeta, ws
      // (p[9]: optional residual-branch gradient added to dx, mmdx_layernorm_bwd_residual)
      if (P(o, 9, ext))
        return mmdx_layernorm_bwd_residual(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                                           (const float*)P(o, 2, ext),
                                           (const float*)P(o, 3, ext),
                                           (const float*)P(o, 4, ext), P(o, 9, ext),
                                           P(o, 5, ext), (float*)P(o, 6, ext),
                                           (float*)P(o, 7, ext), o.f[0], P(o, 8, ext),
                                           (size_t)o.l[1], s);
      return mmdx_layernorm_bwd(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                                (const float*)P(o, 2, ext), (const float*)P(o, 3, ext),
                                (const float*)P(o, 4, ext), P(o, 5, ext), (float*)P(o, 6, ext),
                                (float*)P(o, 7, ext), o.f[0], P(o, 8, ext), (size_t)o.l[1], s);
    case MMDX_OP_LN_FWD_DROP:
      // i: D; l: rows, seed; f: eps, p; p: x, residual, gamma, beta, y, sum_out, mean, rstd,
      // counter, rng
      return mmdx_layernorm_fwd_dropout(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                                        (const float*)P(o, 2, ext), (const float*)P(o, 3, ext),
                                        o.f[0], o.f[1], (uint64_t)o.l[1], (uint64_t*)P(o, 8, ext),
                                        P(o, 4, ext), P(o, 5, ext), (float*)P(o, 6, ext),
                                        (float*)P(o, 7, ext), (uint64_t*)P(o, 9, ext), s);
    case MMDX_OP_LN_BWD_DROP:
      // i: D; l: rows, ws_bytes; f: beta_acc, p; p: xsum, dy, gamma, mean, rstd, dx, dgamma,
      // dbeta, ws, rng, dx_drop
      return mmdx_layernorm_bwd_dropout(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                                        (const float*)P(o, 2, ext), (const float*)P(o, 3, ext),
                                        (const float*)P(o, 4, ext), o.f[1],
                                        (const uint64_t*)P(o, 9, ext), P(o, 5, ext),
                                        P(o, 10, ext), (float*)P(o, 6, ext), (float*)P(o, 7, ext),
                                        o.f[0], P(o, 8, ext), (size_t)o.l[1], s);
    case MMDX_OP_GELU_BWD:  // l: n; p: pre, dy, dx
      return mmdx_gelu_bwd(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], P(o, 2, ext), s);
    case MMDX_OP_BIAS_GRAD:  // i: N; l: M, ws_bytes; f: beta_acc; p: dy, db, ws
      return mmdx_bias_grad(o.dtype, P(o, 0, ext), o.l[0], o.i[0], (float*)P(o, 1, ext),
                            o.f[0], P(o, 2, ext), (size_t)o.l[1], s);
    case MMDX_OP_ADD:  // l: n; p: x, y, out
      return mmdx_add(o.dtype, o.l[0], P(o, 0, ext), P(o, 1, ext), P(o, 2, ext), s);
    case MMDX_OP_DROPOUT_FWD:
      // f: p; l: n, seed, offset; p: x, counter, y, mask
      return mmdx_dropout_fwd(o.dtype, P(o, 0, ext), o.l[0], o.f[0], (uint64_t)o.l[1],
                              (uint64_t)o.l[2], (uint64_t*)P(o, 1, ext), P(o, 2, ext),
                              (uint8_t*)P(o, 3, ext), s);
    case MMDX_OP_DROPOUT_BWD:  // f: p; l: n; p: dy, mask, dx
      return mmdx_dropout_bwd(o.dtype, P(o, 0, ext), (const uint8_t*)P(o, 1, ext), o.l[0],
                              o.f[0], P(o, 2, ext), s);
    case MMDX_OP_AXPBY:  // l: n; f: a, b; p: x, y, out
      return mmdx_axpby(o.l[0], o.f[0], (const float*)P(o, 0, ext), o.f[1],
                        (const float*)P(o, 1, ext), (float*)P(o, 2, ext), s);
    case MMDX_OP_BN_APPLY:
      return mmdx_bn_apply(o.dtype, P(o, 0, ext), P(o, 1, ext), o.l[0], o.i[0],
                           (const float*)P(o, 2, ext), (const float*)P(o, 3, ext), o.i[1],
                           P(o, 4, ext), (uint8_t*)P(o, 5, ext), s);
    default:
      mmdx_set_error("plan: unknown op code %d", o.op);
      return -22;
  }
}

}  // namespace

extern "C" size_t mmdx_plan_op_size(void) { return sizeof(mmdx_plan_op); }

extern "C" int mmdx_plan_run(const mmdx_plan_op* ops, int n_ops, void* const* ext,
                             void* const* events, void* const* streams, int n_streams) {
  if (!ops || n_ops < 0 || !streams || n_streams < 1) {
    mmdx_set_error("plan: bad op list or stream table");
    return -22;
  }
  for (int k = 0; k < n_ops; ++k) {
    if (ops[k].stream < 0 || ops[k].stream >= n_streams) {
      mmdx_set_error("plan: op %d names stream %d of %d", k, ops[k].stream, n_streams);
      return -22;
    }
  }
  for (int k = 0; k < n_ops; ++k) {
    const int rc = run_one(ops[k], ext, events, streams[ops[k].stream]);
    if (rc) return rc;  // the failing op's own message stays in mmdx_last_error()
  }
  return 0;
}
