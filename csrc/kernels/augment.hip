// On-device image augmentation fused with the permutation gather:
// RandomResizedCrop + horizontal flip + per-channel normalise + cast, one pass.
//
// The reference ships no augmentation (its harness data are tabular rows,
// tests/run_ddl.py:80-104); an image loader feeding an MI355X at ~190k
// samples/s cannot run torchvision's per-sample CPU transforms, so the crop
// parameters are drawn ON THE DEVICE from a counter-based hash of
// (seed, sample id): deterministic, independent of rank / world size / batch
// composition, and with no host work or H2D per batch. The parameter draw
// follows torchvision's RandomResizedCrop.get_params (10 attempts of
// (scale, log-uniform ratio), then the centre-crop fallback); resampling is
// bilinear with align_corners=False (torch.nn.functional.interpolate).
//
// Mapping: one thread per output pixel (all channels), 256 pixels per
// workgroup, workgroups of one image contiguous; consecutive lanes write
// consecutive output pixels of each channel plane (coalesced), and read
// neighbouring source pixels (L1/L2 hits).
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;
static_assert(sizeof(CropBox) == 5 * sizeof(int32_t), "CropBox must match the [B, 5] int32 boxes tensor");

__device__ __forceinline__ float unit_uniform(uint64_t seed, uint64_t sample, uint32_t k) {
  const uint64_t z = mix64(seed ^ mix64(sample * 0x9E3779B97F4A7C15ull + k));
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);  // 24 bits -> [0, 1)
}

__device__ CropBox draw_crop(const AugmentSpec& a, uint64_t sample) {
  CropBox b;
  const int H = a.in_h, W = a.in_w;
  const float area = static_cast<float>(H) * static_cast<float>(W);
  const float lr0 = logf(a.ratio_min), lr1 = logf(a.ratio_max);
  bool ok = false;
  for (int t = 0; t < 10 && !ok; ++t) {
    const float target = area * (a.scale_min + (a.scale_max - a.scale_min) * unit_uniform(a.seed, sample, 2 * t));
    const float aspect = expf(lr0 + (lr1 - lr0) * unit_uniform(a.seed, sample, 2 * t + 1));
    const int w = static_cast<int>(rintf(sqrtf(target * aspect)));
    const int h = static_cast<int>(rintf(sqrtf(target / aspect)));
    if (w > 0 && w <= W && h > 0 && h <= H) {
      b.h = h;
      b.w = w;
      b.y = min(static_cast<int>(unit_uniform(a.seed, sample, 20 + 2 * t) * static_cast<float>(H - h + 1)), H - h);
      b.x = min(static_cast<int>(unit_uniform(a.seed, sample, 21 + 2 * t) * static_cast<float>(W - w + 1)), W - w);
      ok = true;
    }
  }
  if (!ok) {  // centre crop with the ratio clamped into [ratio_min, ratio_max]
    const float in_ratio = static_cast<float>(W) / static_cast<float>(H);
    if (in_ratio < a.ratio_min) {
      b.w = W;
      b.h = min(H, max(1, static_cast<int>(rintf(static_cast<float>(W) / a.ratio_min))));
    } else if (in_ratio > a.ratio_max) {
      b.h = H;
      b.w = min(W, max(1, static_cast<int>(rintf(static_cast<float>(H) * a.ratio_max))));
    } else {
      b.w = W;
      b.h = H;
    }
    b.y = (H - b.h) / 2;
    b.x = (W - b.w) / 2;
  }
  b.flip = unit_uniform(a.seed, sample, 40) < a.flip_p ? 1 : 0;
  return b;
}

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  if constexpr (sizeof(T) == 2)
    return bf16_bits_to_f32(*reinterpret_cast<const uint16_t*>(p));
  else
    return static_cast<float>(*p);
}

// One thread per image: draw its crop box (10 attempts of hash + log/exp/sqrt)
// once, instead of once per workgroup of the resampling kernel.
__global__ void __launch_bounds__(kThreads) rrc_boxes_kernel(AugmentSpec a, int64_t batch, RowIndex ri,
                                                            CropBox* __restrict__ boxes) {
  const int64_t img = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (img >= batch) return;
  boxes[img] = draw_crop(a, static_cast<uint64_t>(a.sample_base + source_row(ri, img)));
}

// HWC=1: src rows are [H, W, C]; else [C, H, W]. out: [B, C, OH, OW].
// Each thread produces kPx consecutive output pixels (all channels): 12 * kPx
// independent tap loads in flight per lane (the kernel is latency-bound, one
// pixel per thread left most of each wave's life waiting on memory), the box
// and index math amortised, and one 8 B store per channel when the row allows.
constexpr int kPx = 4;

template <typename Tin, int HWC, int OUT_BF16>
__global__ void __launch_bounds__(kThreads) rrc_kernel(void* __restrict__ dst, const Tin* __restrict__ src,
                                                      AugmentSpec a, int64_t tiles, RowIndex ri, Affine aff,
                                                      const CropBox* __restrict__ boxes) {
  const int64_t img = blockIdx.x / static_cast<uint32_t>(tiles);
  const int64_t t = blockIdx.x - static_cast<uint32_t>(img) * static_cast<uint32_t>(tiles);
  const int64_t srow = source_row(ri, img);
  const CropBox b = boxes[img];  // wave-uniform (scalar) load
  const int opix = a.out_h * a.out_w;
  const int q0 = (static_cast<int>(t) * kThreads + static_cast<int>(threadIdx.x)) * kPx;
  if (q0 >= opix) return;
  const int C = a.channels;
  const int64_t plane = static_cast<int64_t>(a.in_h) * a.in_w;
  const Tin* s = src + srow * plane * C;
  const float fy = static_cast<float>(b.h) / a.out_h, fx = static_cast<float>(b.w) / a.out_w;
  int64_t i00[kPx], i01[kPx], i10[kPx], i11[kPx];
  float wy[kPx], wx[kPx];
#pragma unroll
  for (int k = 0; k < kPx; ++k) {
    const int q = min(q0 + k, opix - 1);  // tail lanes recompute the last pixel (not stored)
    const int oy = q / a.out_w;
    int ox = q - oy * a.out_w;
    if (b.flip) ox = a.out_w - 1 - ox;
    // bilinear, align_corners=False: src = (dst + 0.5) * in/out - 0.5, clamped at 0
    const float sy = fmaxf((static_cast<float>(oy) + 0.5f) * fy - 0.5f, 0.f);
    const float sx = fmaxf((static_cast<float>(ox) + 0.5f) * fx - 0.5f, 0.f);
    const int y0 = min(static_cast<int>(sy), b.h - 1), x0 = min(static_cast<int>(sx), b.w - 1);
    const int y1 = y0 + (y0 < b.h - 1 ? 1 : 0), x1 = x0 + (x0 < b.w - 1 ? 1 : 0);
    wy[k] = sy - static_cast<float>(y0);
    wx[k] = sx - static_cast<float>(x0);
    const int64_t r0 = static_cast<int64_t>(b.y + y0) * a.in_w, r1 = static_cast<int64_t>(b.y + y1) * a.in_w;
    const int64_t c0 = b.x + x0, c1 = b.x + x1;
    i00[k] = r0 + c0;
    i01[k] = r0 + c1;
    i10[k] = r1 + c0;
    i11[k] = r1 + c1;
  }
  const bool vec = (opix % kPx == 0) && (q0 + kPx <= opix);  // 4 contiguous outputs per channel, 8 B aligned
  const int64_t o = img * static_cast<int64_t>(C) * opix + q0;
  for (int c = 0; c < C; ++c) {
    float v[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      float v00, v01, v10, v11;
      if constexpr (HWC) {
        v00 = ld(s + i00[k] * C + c);
        v01 = ld(s + i01[k] * C + c);
        v10 = ld(s + i10[k] * C + c);
        v11 = ld(s + i11[k] * C + c);
      } else {
        const Tin* sc = s + c * plane;
        v00 = ld(sc + i00[k]);
        v01 = ld(sc + i01[k]);
        v10 = ld(sc + i10[k]);
        v11 = ld(sc + i11[k]);
      }
      const float top = v00 + (v01 - v00) * wx[k];
      const float bot = v10 + (v11 - v10) * wx[k];
      v[k] = top + (bot - top) * wy[k];
      if (aff.enabled) v[k] = fmaf(v[k], aff.scale[c], aff.bias[c]);
    }
    const int64_t oc = o + static_cast<int64_t>(c) * opix;
    if constexpr (OUT_BF16) {
      uint16_t* d = static_cast<uint16_t*>(dst) + oc;
      if (vec) {
        *reinterpret_cast<uint2*>(d) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      } else {
        for (int k = 0; k < kPx && q0 + k < opix; ++k) d[k] = f32_to_bf16_bits(v[k]);
      }
    } else {
      float* d = static_cast<float*>(dst) + oc;
      if (vec) {
        *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        for (int k = 0; k < kPx && q0 + k < opix; ++k) d[k] = v[k];
      }
    }
  }
}

template <typename Tin, int HWC>
int launch_rrc(void* dst, int32_t out_dt, const void* src, int64_t batch, const AugmentSpec& a, const RowIndex& ri,
               const Affine& aff, int32_t* boxes_out, hipStream_t st) {
  auto* boxes = reinterpret_cast<CropBox*>(boxes_out);
  hipLaunchKernelGGL(rrc_boxes_kernel, dim3(static_cast<uint32_t>((batch + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, st, a, batch, ri, boxes);
  const int64_t tiles = (static_cast<int64_t>(a.out_h) * a.out_w + kThreads * kPx - 1) / (kThreads * kPx);
  const dim3 grid(static_cast<uint32_t>(batch * tiles));
  if (out_dt == kBF16)
    hipLaunchKernelGGL((rrc_kernel<Tin, HWC, 1>), grid, dim3(kThreads), 0, st, dst, static_cast<const Tin*>(src), a,
                       tiles, ri, aff, boxes);
  else if (out_dt == kF32)
    hipLaunchKernelGGL((rrc_kernel<Tin, HWC, 0>), grid, dim3(kThreads), 0, st, dst, static_cast<const Tin*>(src), a,
                       tiles, ri, aff, boxes);
  else
    return -1;
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int random_resized_crop(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t batch,
                        const AugmentSpec& a, int hwc, const RowIndex& ri, const Affine& aff, int32_t* boxes_out,
                        hipStream_t st) {
  if (batch <= 0) return 0;
  if (boxes_out == nullptr) return -3;  // [batch, 5] int32 device buffer: boxes are drawn there first
  if (a.channels < 1 || a.channels > kMaxAffineChannels || a.in_h < 1 || a.in_w < 1 || a.out_h < 1 || a.out_w < 1)
    return -2;
  if (batch * ((static_cast<int64_t>(a.out_h) * a.out_w + kThreads - 1) / kThreads) >= (int64_t{1} << 31)) return -4;
  switch (in_dt) {
    case kU8:
      return hwc ? launch_rrc<uint8_t, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st)
                 : launch_rrc<uint8_t, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st);
    case kF32:
      return hwc ? launch_rrc<float, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st)
                 : launch_rrc<float, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st);
    case kBF16:
      return hwc ? launch_rrc<uint16_t, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st)
                 : launch_rrc<uint16_t, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, st);
  }
  return -1;
}

}  // namespace ddl
