// The 3x3 / stride-2 max pool's backward gather (the ResNet stem pool, backbone[3], TP:183),
// shared by the pool's own backward kernel (misc.hip) and by the stem BatchNorm backward,
// which reads the pooled gradient through it instead of a materialised dL/d(pool input)
// (norm.hip, mmdx_bn_bwd_pool).  Both round the gathered sum to T, so the fused BN backward
// sees exactly the values the separate pass would have written.
#pragma once
#include "common.h"

namespace mmdx {

template <int VEC> struct ArgPack;  // VEC argmax bytes in one load / store
template <> struct ArgPack<8> { typedef unsigned long long type; };
template <> struct ArgPack<4> { typedef unsigned type; };

template <typename T>
struct Pool3s2Grad {
  typedef typename Vec16<T>::type V;
  static constexpr int VEC = Vec16<T>::N;
  typedef typename ArgPack<VEC>::type A;
  const uint8_t* am;  // [N][P][Q][C] window index of each pooled element's maximum
  const T* dy;        // [N][P][Q][C] gradient of the pooled output
  int H, W, C, p, P, Q;

  // dL/dx at input pixel (n, h, w), channels c .. c+VEC-1: an input pixel lies in at most
  // 2 x 2 windows; their dy vectors and packed argmax bytes are loaded together and summed in
  // ascending window order (the generic pool backward's order)
  __device__ __forceinline__ V at(int n, int h, int w, int c) const {
    const int ph = (h + p) >> 1, qw = (w + p) >> 1;  // the last window that can hold (h, w)
    V g[2][2];
    A a[2][2];
    bool ok[2][2];
#pragma unroll
    for (int dp = 0; dp < 2; ++dp) {
      const int pp = ph - 1 + dp, r = h + p - 2 * pp;
#pragma unroll
      for (int dq = 0; dq < 2; ++dq) {
        const int q = qw - 1 + dq, ss = w + p - 2 * q;
        ok[dp][dq] = pp >= 0 && pp < P && q >= 0 && q < Q && r >= 0 && r < 3 && ss >= 0 &&
                     ss < 3;
        const long o = (((long)n * P + pp) * Q + q) * C + c;
        g[dp][dq] = ok[dp][dq] ? *(const V*)(dy + o) : V{};
        a[dp][dq] = ok[dp][dq] ? *(const A*)(am + o) : (A)0;
      }
    }
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
#pragma unroll
    for (int dp = 0; dp < 2; ++dp)
#pragma unroll
      for (int dq = 0; dq < 2; ++dq) {
        if (!ok[dp][dq]) continue;
        const int tap = (h + p - 2 * (ph - 1 + dp)) * 3 + (w + p - 2 * (qw - 1 + dq));
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          if ((int)((a[dp][dq] >> (8 * j)) & 0xff) == tap) acc[j] += to_f(g[dp][dq][j]);
      }
    V out;
#pragma unroll
    for (int j = 0; j < VEC; ++j) out[j] = from_f<T>(acc[j]);
    return out;
  }
  // the same for NHWC row r = (n*H + h)*W + w (rows < 2^31, checked by mmdx_bn_bwd_pool:
  // 32-bit divisions — a 64-bit one is a long software sequence on the GPU)
  __device__ __forceinline__ V row(long r, int c) const {
    const unsigned ur = (unsigned)r;
    const int w = (int)(ur % (unsigned)W);
    const unsigned t = ur / (unsigned)W;
    const int h = (int)(t % (unsigned)H);
    return at((int)(t / (unsigned)H), h, w, c);
  }
};

// the dense gradient source of the ordinary BN backward
template <typename T>
struct DenseGrad {
  typedef typename Vec16<T>::type V;
  const T* dy;
  int C;
  __device__ __forceinline__ V row(long r, int c) const {  // streaming (nontemporal) load
    return __builtin_nontemporal_load((const V*)(dy + r * C + c));
  }
};

// dy with a 1-bit ReLU mask applied on the fly ([rows][C / VEC] bytes, mmdx_bn_fwd_ex): the
// gradient that leaves a residual unit through its identity path, read by the downsample
// BatchNorm's backward without being materialised (mmdx_bn_bwd_masked_dy)
template <typename T>
struct MaskedGrad {
  typedef typename Vec16<T>::type V;
  static constexpr int VEC = Vec16<T>::N;
  const T* dy;
  const uint8_t* mask;
  int C;
  __device__ __forceinline__ V row(long r, int c) const {
    V v = *(const V*)(dy + r * C + c);
    const unsigned b = mask[r * (C / VEC) + c / VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e)
      if (!((b >> e) & 1u)) v[e] = from_f<T>(0.f);
    return v;
  }
};

}  // namespace mmdx
