// Host data step on the GPU: Pillow-exact antialiased bicubic resize + SigLIP rescale/normalise.
//
// Replaces the per-image pixel work of XrayTextPairDataset.__getitem__
// (Stage1/train_projection_stage1.py:97-99: `.convert('RGB').resize((S, S))` then
// `processor(images=...)`), which the reference runs on host worker processes.
// The JPEG decode stays on the host; the decoded uint8 image (1 channel for a
// greyscale X-ray, 3 otherwise) is what crosses PCIe, a fraction of the float32
// pixel_values.
//
// Semantics (Pillow src/libImaging/Resample.c, restated in oracle/image_ref.py):
//   weights   precompute_coeffs + normalize_coeffs_8bpc (host, below, in double,
//             no FP contraction, as Pillow's C);
//   pass 1    horizontal, every source row -> uint8 [h][S][c]:
//             clip8((2^21 + sum_t src[lo + t] * k[t]) >> 22) in int32;
//   pass 2    vertical on that intermediate, same rounding;
//   normalise a [3][256] table of the output type, one row per RGB channel (rescale 1/255
//             in float64 -> float32, (x - mean[c]) / std[c] in float32, then bf16 RNE), built
//             by the caller.
// Both passes are integer arithmetic: results are bit-identical to Pillow.
//
// Kernels (HBM-bound byte work, no MFMA): pass 1 stages one source row per
// workgroup in LDS (coalesced), then every lane produces outputs from LDS;
// pass 2 reads S consecutive intermediate bytes per tap row (coalesced) and
// writes the three planar output rows contiguously.
#include <math.h>

#include "common.h"
#include "ptk_internal.h"
#include "../../include/ptk.h"

namespace ptk {

constexpr int IMG_PREC = 22;   // Resample.c PRECISION_BITS = 32 - 8 - 2

PTK_DEV unsigned char clip8(int acc) {
  const int v = acc >> IMG_PREC;   // arithmetic shift, as Pillow's clip8 table index
  return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

__global__ void __launch_bounds__(256) resize_h_kernel(const uint8_t* __restrict__ src,
                                                       const int32_t* __restrict__ coefs,
                                                       const ptk_image_desc* __restrict__ desc, int S,
                                                       uint8_t* __restrict__ tmp) {
  extern __shared__ unsigned char row[];
  const ptk_image_desc d = desc[blockIdx.y];
  const int y = blockIdx.x;
  if (y >= d.h) return;
  const int rb = d.w * d.c;
  const uint8_t* s = src + d.src_off + (long)y * rb;
  for (int i = threadIdx.x; i < rb; i += 256) row[i] = s[i];
  __syncthreads();
  const int32_t* bh = coefs + d.coef_off;
  const int32_t* kh = bh + 2 * S;
  uint8_t* t = tmp + d.tmp_off + (long)y * S * d.c;
  const int c = d.c;
  for (int idx = threadIdx.x; idx < S * c; idx += 256) {
    const int o = c == 1 ? idx : idx / 3, ch = idx - o * c;
    const int lo = bh[2 * o], n = bh[2 * o + 1];
    const int32_t* k = kh + (long)o * d.kh;
    const unsigned char* r = row + lo * c + ch;
    int acc = 1 << (IMG_PREC - 1);
    for (int j = 0; j < n; ++j) acc += (int)r[j * c] * k[j];
    t[idx] = clip8(acc);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) resize_v_kernel(const int32_t* __restrict__ coefs,
                                                       const ptk_image_desc* __restrict__ desc, int S,
                                                       const uint8_t* __restrict__ tmp, const T* __restrict__ lut,
                                                       T* __restrict__ out) {
  __shared__ T tab[3][256];
  tab[0][threadIdx.x] = lut[threadIdx.x];
  tab[1][threadIdx.x] = lut[256 + threadIdx.x];
  tab[2][threadIdx.x] = lut[512 + threadIdx.x];
  __syncthreads();
  const ptk_image_desc d = desc[blockIdx.y];
  const int yo = blockIdx.x, c = d.c;
  const int32_t* bv = coefs + d.coef_off + 2 * S + (long)S * d.kh;
  const int lo = bv[2 * yo], n = bv[2 * yo + 1];
  const int32_t* k = bv + 2 * S + (long)yo * d.kv;
  const uint8_t* t = tmp + d.tmp_off + (long)lo * S * c;
  const long plane = (long)S * S;
  T* o = out + (long)blockIdx.y * 3 * plane + (long)yo * S;
  for (int idx = threadIdx.x; idx < S * c; idx += 256) {
    const int ch = c == 1 ? 0 : idx / S, xo = idx - ch * S;
    const uint8_t* p = t + xo * c + ch;
    int acc = 1 << (IMG_PREC - 1);
    for (int j = 0; j < n; ++j) acc += (int)p[(long)j * S * c] * k[j];
    const unsigned char v = clip8(acc);
    if (c == 1) {
      o[xo] = tab[0][v];
      o[plane + xo] = tab[1][v];
      o[2 * plane + xo] = tab[2][v];
    } else {
      o[ch * plane + xo] = tab[ch][v];
    }
  }
}

}  // namespace ptk

using namespace ptk;

extern "C" int ptk_resize_ksize(int in_size, int out_size) {
  if (in_size <= 0 || out_size <= 0) return set_error("resize: sizes %d -> %d", in_size, out_size);
  const double scale = (double)in_size / out_size;
  const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
  return (int)ceil(support) * 2 + 1;
}

extern "C" int ptk_resize_coeffs(int in_size, int out_size, int32_t* bounds, int32_t* coeffs) {
#pragma clang fp contract(off)
  const int ksize = ptk_resize_ksize(in_size, out_size);
  if (ksize < 0) return ksize;
  const double scale = (double)in_size / out_size;   // Pillow: (double)(in1 - in0) / outSize
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double ss = 1.0 / filterscale;
  auto bicubic = [](double x) {   // Resample.c bicubic_filter, a = -0.5
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
  };
  double w[1 << 12];
  if (ksize > (1 << 12)) return set_error("resize: %d -> %d needs %d taps", in_size, out_size, ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      w[x] = bicubic((x + xmin - center + 0.5) * ss);
      ww += w[x];
    }
    int32_t* k = coeffs + (long)xx * ksize;
    for (int x = 0; x < ksize; ++x) {
      double v = 0.0;
      if (x < xmax) v = ww != 0.0 ? w[x] / ww : w[x];
      k[x] = v < 0 ? (int32_t)(-0.5 + v * (1 << IMG_PREC)) : (int32_t)(0.5 + v * (1 << IMG_PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

extern "C" int ptk_image_preprocess(const uint8_t* src, const int32_t* coefs, const ptk_image_desc* desc, int n,
                                    int max_h, int max_row_bytes, int out_size, const void* lut, int out_f32,
                                    uint8_t* tmp, void* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n < 0 || max_h < 0 || out_size <= 0) return set_error("image_preprocess: n %d max_h %d size %d", n, max_h, out_size);
  if (max_row_bytes <= 0 || max_row_bytes > 65536) return set_error("image_preprocess: row bytes %d", max_row_bytes);
  if (n == 0 || max_h == 0) return 0;
  if (n > 65535) return set_error("image_preprocess: %d images per call", n);
  hipLaunchKernelGGL(resize_h_kernel, dim3(max_h, n), dim3(256), max_row_bytes, st, src, coefs, desc, out_size, tmp);
  if (out_f32)
    hipLaunchKernelGGL(resize_v_kernel<float>, dim3(out_size, n), dim3(256), 0, st, coefs, desc, out_size, tmp,
                       (const float*)lut, (float*)out);
  else
    hipLaunchKernelGGL(resize_v_kernel<bf16_t>, dim3(out_size, n), dim3(256), 0, st, coefs, desc, out_size, tmp,
                       (const bf16_t*)lut, (bf16_t*)out);
  return hipGetLastError() == hipSuccess ? 0 : set_error("image_preprocess launch failed");
}
