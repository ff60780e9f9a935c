// Batched image preprocessing on the GPU, bit-exact with the reference's CPU transform
// image_transfom_into_tensor (training_pipeline.py:112-119): torchvision Resize(256,
// antialias=True) on a PIL image = PIL's ImagingResample with the bilinear filter (two
// separable fixed-point passes, horizontal first, 22-bit coefficients, uint8 intermediate
// clipped after each pass), CenterCrop(224), ToTensor (/255), gray -> RGB repeat,
// Normalize(ImageNet mean/std).  JPEG decode stays on the host (PIL, as in the reference,
// TP:146).  Only the 224x224 crop window of the resized image is computed: every output
// value of a separable resample depends on its own row/column coefficients only, so the
// window's values are exactly those of the full resize.
//
// The host (mmdx.preprocess) computes the per-image coefficient tables in double precision
// with PIL's formulas and uploads them with the packed uint8 pixels.
#include <algorithm>

#include "common.h"
#include "../../include/mmdx.h"

namespace mmdx {

constexpr int PRE_BITS = 22;  // PIL PRECISION_BITS = 32 - 8 - 2

__device__ __forceinline__ int pil_clip8(int v) {
  if (v >= (1 << PRE_BITS << 8)) return 255;
  if (v <= 0) return 0;
  return v >> PRE_BITS;
}

// Horizontal pass: temp[b][r][j][c] = clip8(sum_x src[row0 + r][xmin_j + x][c] * kh_j[x]) for
// the crop columns j of the resized image (or a straight copy when the width is unchanged).
__global__ void pre_horizontal_kernel(const uint8_t* __restrict__ px,
                                      const mmdx_img_desc* __restrict__ descs,
                                      const int* __restrict__ coef, int out_w,
                                      uint8_t* __restrict__ temp) {
  const mmdx_img_desc d = descs[blockIdx.y];
  const int r = blockIdx.x;
  if (r >= d.trows) return;
  const int y = d.trow0 + r;  // source row
  const uint8_t* src = px + d.src_off + (long)y * d.w * d.c;
  uint8_t* dst = temp + d.temp_off + (long)r * out_w * d.c;
  for (int e = threadIdx.x; e < out_w * d.c; e += blockDim.x) {
    const int j = e / d.c, ch = e - j * d.c;
    if (!d.need_h) {
      dst[e] = src[(d.left + j) * d.c + ch];
      continue;
    }
    const int* k = coef + d.kh_off + (long)j * (d.ksize_h + 2);
    const int xmin = k[0], xmax = k[1];
    int ss = 1 << (PRE_BITS - 1);
    for (int x = 0; x < xmax; ++x) ss += (int)src[(xmin + x) * d.c + ch] * k[2 + x];
    dst[e] = (uint8_t)pil_clip8(ss);
  }
}

// Vertical pass + crop + ToTensor + gray->RGB + Normalize -> out [B][3][out_h][out_w] fp32.
__global__ void pre_vertical_kernel(const uint8_t* __restrict__ temp,
                                    const mmdx_img_desc* __restrict__ descs,
                                    const int* __restrict__ coef, int out_h, int out_w,
                                    float* __restrict__ out) {
  const mmdx_img_desc d = descs[blockIdx.y];
  const int i = blockIdx.x;  // output row
  const float mean[3] = {0.485f, 0.456f, 0.406f};
  const float stdv[3] = {0.229f, 0.224f, 0.225f};
  const uint8_t* t = temp + d.temp_off;
  for (int j = threadIdx.x; j < out_w; j += blockDim.x) {
    for (int ch = 0; ch < d.c; ++ch) {
      int v;
      if (d.need_v) {
        const int* k = coef + d.kv_off + (long)i * (d.ksize_v + 2);
        const int ymin = k[0], ymax = k[1];  // ymin relative to trow0
        int ss = 1 << (PRE_BITS - 1);
        for (int y = 0; y < ymax; ++y) ss += (int)t[((long)(ymin + y) * out_w + j) * d.c + ch] * k[2 + y];
        v = pil_clip8(ss);
      } else {
        v = t[((long)(d.top + i - d.trow0) * out_w + j) * d.c + ch];
      }
      const float f = (float)v / 255.f;  // ToTensor: float(u8) / 255
      for (int oc = (d.c == 1 ? 0 : ch); oc < (d.c == 1 ? 3 : ch + 1); ++oc)
        out[(((long)blockIdx.y * 3 + oc) * out_h + i) * out_w + j] = (f - mean[oc]) / stdv[oc];
    }
  }
}

}  // namespace mmdx

using namespace mmdx;

extern "C" size_t mmdx_img_desc_size(void) { return sizeof(mmdx_img_desc); }

extern "C" int mmdx_image_preprocess(const uint8_t* pixels, const mmdx_img_desc* descs, int B,
                                     const int* coef, int max_trows, int out_h, int out_w,
                                     uint8_t* temp, float* out, void* stream) {
  MMDX_CHECK_ARG(B > 0 && pixels && descs && coef && temp && out && out_h > 0 && out_w > 0,
                 "image preprocess: bad args");
  MMDX_CHECK_ARG(max_trows > 0 && B <= 65535, "image preprocess: bad batch geometry");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(pre_horizontal_kernel, dim3(max_trows, B), dim3(256), 0, st, pixels, descs,
                     coef, out_w, temp);
  hipLaunchKernelGGL(pre_vertical_kernel, dim3(out_h, B), dim3(256), 0, st, temp, descs, coef,
                     out_h, out_w, out);
  MMDX_LAUNCH_CHECK();
  return 0;
}
