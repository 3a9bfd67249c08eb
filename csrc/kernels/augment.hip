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
// Mapping: one workgroup per (image, band of R output rows). The band's source
// rows -- at most ceil((R-1) * in_h / out_h) + 3 rows of the crop, every
// channel, only the crop's columns -- are first copied into LDS with aligned
// 16 B loads (all of a lane's loads issued before its LDS writes), then every
// bilinear tap is an LDS read. The earlier form read each tap straight from
// global memory: 48 one-byte VMEM instructions per lane for 4 uint8 pixels,
// which PMC showed to be memory-instruction-issue bound (SQ_WAIT_INST_ANY
// ~2.6x the active cycles, archive/profiles/r1_augment/). Consecutive lanes write
// consecutive output pixels of each channel plane (a wave store covers 128 B of
// bf16 / 256 B of f32). A geometry whose band does not fit the LDS budget runs
// the same kernel with the taps read from global memory.
#include <algorithm>

#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;
constexpr int kBandMaxRows = 16;
constexpr int64_t kBandLdsBudget = 32 * 1024;  // 4-5 workgroups (16-20 waves) per CU
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
  const int64_t key = a.sample_ids != nullptr ? a.sample_ids[img] : source_row(ri, img);
  boxes[img] = draw_crop(a, static_cast<uint64_t>(a.sample_base + key));
}

// Division by a runtime divisor d that is uniform across the workgroup, for
// dividends with w * d < 2^32 (LDS chunk and pixel indices here): with
// m = ceil(2^32 / d), floor(w / d) = umulhi(w, m) exactly in that range (the
// rounding error of m is below 1 / d). Two VALU instructions instead of the
// ~15 of a generic 32-bit udiv; m is computed once per workgroup.
struct FastDiv {
  uint32_t d, m;
  __device__ __forceinline__ explicit FastDiv(uint32_t d_) : d(d_), m(d_ > 1 ? static_cast<uint32_t>(((1ull << 32) + d_ - 1) / d_) : 0u) {}
  __device__ __forceinline__ uint32_t div(uint32_t w) const { return d > 1 ? __umulhi(w, m) : w; }
};

// Bilinear source coordinate of output index o, align_corners=False:
// src = (dst + 0.5) * in/out - 0.5, clamped at 0. The band bounds and the taps
// both come from this one function, so they agree bit for bit.
__device__ __forceinline__ float src_coord(int o, float f) {
  return fmaxf((static_cast<float>(o) + 0.5f) * f - 0.5f, 0.f);
}

// Each thread produces kPx consecutive output pixels of the band (all
// channels): the box and index math are amortised, 4 * kPx independent taps
// per channel are in flight, and one 8 B (bf16) / 16 B (f32) store per
// channel when the output row allows. tap(c, y, x) reads crop-relative source
// pixel (y, x) of channel c.
constexpr int kPx = 4;

template <int OUT_BF16, typename Tap>
__device__ __forceinline__ void resample_band(void* __restrict__ dst, int64_t img, const AugmentSpec& a,
                                              const CropBox& b, int oy0, int oy1, const Affine& aff, Tap tap) {
  const int ow = a.out_w, C = a.channels;
  const int64_t opix = static_cast<int64_t>(a.out_h) * ow;
  const int n = (oy1 - oy0) * ow;
  const float fy = static_cast<float>(b.h) / a.out_h, fx = static_cast<float>(b.w) / a.out_w;
  const bool vec_ok = (ow % kPx) == 0;  // band rows start 4-aligned in the plane: aligned vector stores
  const FastDiv div_ow(static_cast<uint32_t>(ow));  // q < 16 * ow, out_w <= 8192 (host check)
  for (int q0 = static_cast<int>(threadIdx.x) * kPx; q0 < n; q0 += kThreads * kPx) {
    int ya[kPx], yb[kPx], xa[kPx], xb[kPx];
    float wy[kPx], wx[kPx];
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      const int q = min(q0 + k, n - 1);  // tail lanes recompute the last pixel (not stored)
      const int r = static_cast<int>(div_ow.div(static_cast<uint32_t>(q)));
      int ox = q - r * ow;
      if (b.flip) ox = ow - 1 - ox;
      const float sy = src_coord(oy0 + r, fy), sx = src_coord(ox, fx);
      const int y0 = min(static_cast<int>(sy), b.h - 1), x0 = min(static_cast<int>(sx), b.w - 1);
      ya[k] = y0;
      yb[k] = y0 + (y0 < b.h - 1 ? 1 : 0);
      xa[k] = x0;
      xb[k] = x0 + (x0 < b.w - 1 ? 1 : 0);
      wy[k] = sy - static_cast<float>(y0);
      wx[k] = sx - static_cast<float>(x0);
    }
    const bool vec = vec_ok && (q0 + kPx <= n);
    const int64_t o = img * C * opix + static_cast<int64_t>(oy0) * ow + q0;
    for (int c = 0; c < C; ++c) {
      float v[kPx];
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const float v00 = tap(c, ya[k], xa[k]), v01 = tap(c, ya[k], xb[k]);
        const float v10 = tap(c, yb[k], xa[k]), v11 = tap(c, yb[k], xb[k]);
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
          for (int k = 0; k < kPx && q0 + k < n; ++k) d[k] = f32_to_bf16_bits(v[k]);
        }
      } else {
        float* d = static_cast<float*>(dst) + oc;
        if (vec) {
          *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          for (int k = 0; k < kPx && q0 + k < n; ++k) d[k] = v[k];
        }
      }
    }
  }
}

// Fast form of resample_band over an LDS band whose rows all start at the same offset `head` within their
// 16 B chunk (row pitch and plane size multiples of 16 B: every standard image geometry). A wave covers
// 64 * kCpl consecutive output columns of one output row per step (kCpl adjacent columns per lane), its 4
// waves take every 4th row of the band. The horizontal taps (x0, x1, weight) of a lane's columns are
// computed once per band and held in registers (kColGroups groups: out_w <= 256 in one pass); the vertical
// ones once per row and wave. A half-wave's byte taps then span 32 * kCpl * fx bytes of one LDS row
// (23 dwords at fx = 1.43: no bank conflicts for CHW rows; the row-major form's 4 pixels per lane spanned
// 128 * fx bytes, up to 2-way CHW / 4-way HWC), and a lane stores its kCpl values of a channel in one
// 4 B (bf16) / 8 B (f32) store. Against the row-major form on one box: 41.1 vs 44.5 us (CHW), 38.8 vs
// 44.4 us (HWC) per 256-image batch; the HBM-resident loader with augmentation, whose consumer kernel runs
// next to it, unchanged (4.78-4.81M vs 4.68-4.89M samples/s). One column per lane (2 B stores) was as fast
// in isolation but 4.5% slower in that loader; 4 per lane doubled the CHW time (profiles/r5_configs/).
// uint8 rows read tap x0 + 1 even at the crop's right edge, with its weight zeroed there:
// v00 + (v01 - v00) * 0 == v00 exactly, as the clamped tap gives (a finite garbage byte times zero), and
// the two taps of a row are one address with an immediate offset. Same float math in the same order as
// resample_band: bit-identical output.
constexpr int kCpl = 2;        // adjacent output columns per lane
constexpr int kColGroups = 2;  // groups of 64 * kCpl columns held in registers: out_w <= 256 per pass
static_assert(kCpl == 2 || kCpl == 4, "the vector stores below pack 2 or 4 values");

template <int OUT_BF16, typename Tin, int HWC, int NC>
__device__ __forceinline__ void resample_band_cols(void* __restrict__ dst, int64_t img, const AugmentSpec& a,
                                                   const CropBox& b, int oy0, int oy1, const Affine& aff,
                                                   const uint8_t* __restrict__ lds, uint32_t head, uint32_t stride,
                                                   uint32_t nrows, int ylo) {
  constexpr uint32_t kSz = static_cast<uint32_t>(sizeof(Tin));
  constexpr bool kEdgeByWeight = sizeof(Tin) == 1;  // garbage taps are finite only for uint8
  constexpr int kWaves = kThreads / 64;
  constexpr int kGw = 64 * kCpl;  // columns per group
  constexpr int kC = NC > 0 ? NC : kMaxAffineChannels;
  const int ow = a.out_w;
  const int C = NC > 0 ? NC : a.channels;
  const uint32_t cin = HWC ? static_cast<uint32_t>(C) : 1u;
  const uint32_t cstep = HWC ? kSz : nrows * stride;  // LDS bytes from one channel to the next
  const int64_t opix = static_cast<int64_t>(a.out_h) * ow;
  const float fy = static_cast<float>(b.h) / a.out_h, fx = static_cast<float>(b.w) / a.out_w;
  const int lane = static_cast<int>(threadIdx.x & 63u);
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int64_t img_o = img * C * opix;
  const bool pair_stores = (ow % kCpl) == 0;  // every lane's first column then sits at an aligned offset
  for (int cg0 = 0; cg0 < ow; cg0 += kGw * kColGroups) {
    const int ng = min(kColGroups, (ow - cg0 + kGw - 1) / kGw);  // uniform
    uint32_t xa[kColGroups][kCpl], xb[kColGroups][kCpl];
    float wx[kColGroups][kCpl];
#pragma unroll
    for (int g = 0; g < kColGroups; ++g) {
#pragma unroll
      for (int j = 0; j < kCpl; ++j) {
        int sxo = min(cg0 + kGw * g + kCpl * lane + j, ow - 1);
        if (b.flip) sxo = ow - 1 - sxo;
        const float sx = src_coord(sxo, fx);
        const int x0 = min(static_cast<int>(sx), b.w - 1);
        const bool edge = x0 >= b.w - 1;
        wx[g][j] = kEdgeByWeight && edge ? 0.f : sx - static_cast<float>(x0);
        xa[g][j] = static_cast<uint32_t>(x0) * cin * kSz + head;
        xb[g][j] = kEdgeByWeight ? xa[g][j] + cin * kSz
                                 : static_cast<uint32_t>(x0 + (edge ? 0 : 1)) * cin * kSz + head;
      }
    }
    for (int r = oy0 + wave; r < oy1; r += kWaves) {  // wave-uniform
      const float sy = src_coord(r, fy);
      const int y0 = min(static_cast<int>(sy), b.h - 1);
      const int y1 = y0 + (y0 < b.h - 1 ? 1 : 0);
      const float wy = sy - static_cast<float>(y0);
      const uint32_t ra = static_cast<uint32_t>(y0 - ylo) * stride;
      const uint32_t rb = static_cast<uint32_t>(y1 - ylo) * stride;
      const int64_t orow = img_o + static_cast<int64_t>(r) * ow + cg0 + kCpl * lane;
#pragma unroll
      for (int g = 0; g < kColGroups; ++g) {
        if (g >= ng) break;
        const int col = cg0 + kGw * g + kCpl * lane;  // this lane's first column
        if (col >= ow) continue;
        const int64_t o = orow + kGw * g;
        float v[kC][kCpl];
#pragma unroll
        for (int c = 0; c < kC; ++c) {  // all taps of all channels issued before any store
          if (NC == 0 && c >= C) break;
          const uint8_t* la = lds + (static_cast<uint32_t>(c) * cstep + ra);
          const uint8_t* lb = lds + (static_cast<uint32_t>(c) * cstep + rb);
#pragma unroll
          for (int j = 0; j < kCpl; ++j) {
            const float v00 = ld(reinterpret_cast<const Tin*>(la + xa[g][j]));
            const float v01 = ld(reinterpret_cast<const Tin*>(la + xb[g][j]));
            const float v10 = ld(reinterpret_cast<const Tin*>(lb + xa[g][j]));
            const float v11 = ld(reinterpret_cast<const Tin*>(lb + xb[g][j]));
            const float top = v00 + (v01 - v00) * wx[g][j];
            const float bot = v10 + (v11 - v10) * wx[g][j];
            v[c][j] = top + (bot - top) * wy;
          }
        }
#pragma unroll
        for (int c = 0; c < kC; ++c) {
          if (NC == 0 && c >= C) break;
          float y[kCpl];
#pragma unroll
          for (int j = 0; j < kCpl; ++j)  // uint8 taps give v >= +0, and fma(v, 1, 0) == v for those
            y[j] = kEdgeByWeight ? fmaf(v[c][j], aff.enabled ? aff.scale[c] : 1.f, aff.enabled ? aff.bias[c] : 0.f)
                                 : (aff.enabled ? fmaf(v[c][j], aff.scale[c], aff.bias[c]) : v[c][j]);
          const int64_t oc = o + static_cast<int64_t>(c) * opix;
          if (pair_stores && col + kCpl <= ow) {
            if constexpr (OUT_BF16) {
              if constexpr (kCpl == 2)
                *reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(dst) + oc) = pack_bf16x2(y[0], y[1]);
              else
                *reinterpret_cast<uint2*>(static_cast<uint16_t*>(dst) + oc) =
                    make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
            } else {
              if constexpr (kCpl == 2)
                *reinterpret_cast<float2*>(static_cast<float*>(dst) + oc) = make_float2(y[0], y[1]);
              else
                *reinterpret_cast<float4*>(static_cast<float*>(dst) + oc) = make_float4(y[0], y[1], y[2], y[3]);
            }
          } else {
#pragma unroll
            for (int j = 0; j < kCpl; ++j) {
              if (col + j >= ow) break;
              if constexpr (OUT_BF16)
                static_cast<uint16_t*>(dst)[oc + j] = f32_to_bf16_bits(y[j]);
              else
                static_cast<float*>(dst)[oc + j] = y[j];
            }
          }
        }
      }
    }
  }
}

// HWC=1: src rows are [H, W, C]; else [C, H, W]. out: [B, C, OH, OW].
// LDS layout: (plane p, band row r) rows of `stride` bytes; row (p, r) holds
// the 16 B-aligned global chunks covering the crop's span of that source row,
// which therefore starts head(p, r) = (global address & 15) bytes into it.
template <typename Tin, int HWC, int OUT_BF16>
__global__ void __launch_bounds__(kThreads) rrc_band_kernel(void* __restrict__ dst, const Tin* __restrict__ src,
                                                           AugmentSpec a, int32_t bands, int32_t band_rows,
                                                           int32_t lds_cap, RowIndex ri, Affine aff,
                                                           const CropBox* __restrict__ boxes) {
  extern __shared__ uint4 lds4[];
  const uint32_t img = blockIdx.x / static_cast<uint32_t>(bands);
  const int band = static_cast<int>(blockIdx.x - img * static_cast<uint32_t>(bands));
  const int64_t srow = source_row(ri, img);
  const CropBox b = boxes[img];  // wave-uniform (scalar) load
  const int oy0 = band * band_rows, oy1 = min(oy0 + band_rows, a.out_h);
  const int C = a.channels;
  constexpr int kSz = static_cast<int>(sizeof(Tin));
  const int planes = HWC ? 1 : C, cin = HWC ? C : 1;
  const int64_t plane_elems = static_cast<int64_t>(a.in_h) * a.in_w;
  const int64_t row_pitch = static_cast<int64_t>(a.in_w) * cin;  // elements
  const Tin* s = src + srow * plane_elems * C;

  const float fy = static_cast<float>(b.h) / a.out_h;
  const int ylo = min(static_cast<int>(src_coord(oy0, fy)), b.h - 1);
  const int ylast = min(static_cast<int>(src_coord(oy1 - 1, fy)), b.h - 1);
  const uint32_t nrows = static_cast<uint32_t>(ylast + (ylast < b.h - 1 ? 1 : 0) - ylo + 1);
  // 16 B chunks per LDS row: the crop span (b.w pixels) starting anywhere in a chunk
  const uint32_t cpr = (15u + static_cast<uint32_t>(b.w * cin * kSz) + 15u) >> 4;
  const uint32_t stride = cpr << 4;

  if (static_cast<int64_t>(planes) * nrows * stride > lds_cap) {  // taps from global memory
    resample_band<OUT_BF16>(dst, img, a, b, oy0, oy1, aff, [&](int c, int y, int x) {
      const int p = HWC ? 0 : c, ci = HWC ? c : 0;
      return ld(s + p * plane_elems + (b.y + y) * row_pitch + static_cast<int64_t>(b.x + x) * cin + ci);
    });
    return;
  }

  // ---- stage the band: crop rows ylo .. ylo+nrows-1 of every plane, 16 B chunks
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s);
  const uintptr_t img_lo = reinterpret_cast<uintptr_t>(s);
  const uintptr_t img_hi = img_lo + static_cast<uintptr_t>(plane_elems * C * kSz);
  const uintptr_t band_base =
      img_lo + static_cast<uintptr_t>(((b.y + ylo) * row_pitch + static_cast<int64_t>(b.x) * cin) * kSz);
  const uintptr_t plane_b = static_cast<uintptr_t>(plane_elems * kSz), pitch_b = static_cast<uintptr_t>(row_pitch * kSz);
  const uint32_t total = static_cast<uint32_t>(planes) * nrows * cpr;
  constexpr int kIlp = 4;
  const FastDiv div_cpr(cpr), div_rows(nrows);  // total <= lds_cap / 16 = 2048 chunks
  for (uint32_t w0 = threadIdx.x; w0 < total; w0 += kIlp * kThreads) {
    uint4 v[kIlp];
#pragma unroll
    for (int k = 0; k < kIlp; ++k) {
      const uint32_t w = w0 + k * kThreads;
      if (w < total) {
        const uint32_t pr = div_cpr.div(w), ch = w - pr * cpr;
        const uint32_t p = div_rows.div(pr), r = pr - p * nrows;
        const uintptr_t row = band_base + p * plane_b + r * pitch_b;
        const uintptr_t g = (row & ~static_cast<uintptr_t>(15)) + 16u * ch;
        // addressed off the kernel argument (not an integer round trip) so the
        // compiler keeps the global address space: global_load_dwordx4, not flat
        const uint8_t* gp = sb + static_cast<intptr_t>(g - img_lo);
        if (g >= img_lo && g + 16 <= img_hi) {
          v[k] = *reinterpret_cast<const uint4*>(gp);
        } else {  // chunk straddles the image bounds: the bytes outside are never sampled
          uint32_t wv[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (g + j >= img_lo && g + j < img_hi) wv[j >> 2] |= static_cast<uint32_t>(gp[j]) << ((j & 3) * 8);
          v[k] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kIlp; ++k)
      if (w0 + k * kThreads < total) lds4[w0 + k * kThreads] = v[k];
  }
  __syncthreads();

  const uint8_t* lds = reinterpret_cast<const uint8_t*>(lds4);
  // low bits of the per-row global addresses (mod 2^32 is enough for & 15)
  const uint32_t base_lo = static_cast<uint32_t>(band_base);
  const uint32_t plane_lo = static_cast<uint32_t>(plane_b), pitch_lo = static_cast<uint32_t>(pitch_b);
  if ((pitch_lo & 15u) == 0 && (planes == 1 || (plane_lo & 15u) == 0)) {
    // every LDS row starts `base_lo & 15` bytes into its first chunk (kernel-uniform branch)
    if (a.channels == 3)
      resample_band_cols<OUT_BF16, Tin, HWC, 3>(dst, img, a, b, oy0, oy1, aff, lds, base_lo & 15u, stride, nrows, ylo);
    else
      resample_band_cols<OUT_BF16, Tin, HWC, 0>(dst, img, a, b, oy0, oy1, aff, lds, base_lo & 15u, stride, nrows, ylo);
    return;
  }
  resample_band<OUT_BF16>(dst, img, a, b, oy0, oy1, aff, [&](int c, int y, int x) {
    const uint32_t p = HWC ? 0u : static_cast<uint32_t>(c);
    const uint32_t ci = HWC ? static_cast<uint32_t>(c) : 0u;
    const uint32_t r = static_cast<uint32_t>(y - ylo);
    const uint32_t head = (base_lo + p * plane_lo + r * pitch_lo) & 15u;
    const uint32_t off = (p * nrows + r) * stride + head + (static_cast<uint32_t>(x) * cin + ci) * kSz;
    return ld(reinterpret_cast<const Tin*>(lds + off));
  });
}

// Band height and LDS allocation for the worst case (crop = whole image):
// rows <= ceil((R-1) * in_h / out_h) + 3, each row the 16 B chunks covering
// in_w * cin elements that may start anywhere in a chunk.
struct BandPlan {
  int32_t rows;
  int64_t lds;  // 0: taps from global memory
};

BandPlan plan_band(const AugmentSpec& a, int hwc, int elem, int path) {
  const int planes = hwc ? 1 : a.channels, cin = hwc ? a.channels : 1;
  const int64_t stride = (static_cast<int64_t>(a.in_w) * cin * elem + 15 + 15) / 16 * 16;
  for (int R = kBandMaxRows; R >= 1 && path != 2; R /= 2) {
    const int64_t rows =
        std::min<int64_t>((static_cast<int64_t>(R - 1) * a.in_h + a.out_h - 1) / a.out_h + 3, a.in_h + 1);
    const int64_t lds = planes * rows * stride;
    if (lds <= kBandLdsBudget) return {R, lds};
  }
  return {kBandMaxRows, 0};
}

template <typename Tin, int HWC>
int launch_rrc(void* dst, int32_t out_dt, const void* src, int64_t batch, const AugmentSpec& a, const RowIndex& ri,
               const Affine& aff, int32_t* boxes_out, int path, hipStream_t st) {
  const BandPlan pl = plan_band(a, HWC, static_cast<int>(sizeof(Tin)), path);
  if (path == 1 && pl.lds == 0) return -5;  // LDS path requested but the geometry does not fit the budget
  const int64_t bands = (a.out_h + pl.rows - 1) / pl.rows;
  if (batch * bands >= (int64_t{1} << 31)) return -4;
  auto* boxes = reinterpret_cast<CropBox*>(boxes_out);
  hipLaunchKernelGGL(rrc_boxes_kernel, dim3(static_cast<uint32_t>((batch + kThreads - 1) / kThreads)), dim3(kThreads),
                     0, st, a, batch, ri, boxes);
  const dim3 grid(static_cast<uint32_t>(batch * bands));
  const auto* s = static_cast<const Tin*>(src);
  const size_t lds = static_cast<size_t>(pl.lds);
  const int32_t nb = static_cast<int32_t>(bands), cap = static_cast<int32_t>(pl.lds);
  if (out_dt == kBF16)
    hipLaunchKernelGGL((rrc_band_kernel<Tin, HWC, 1>), grid, dim3(kThreads), lds, st, dst, s, a, nb, pl.rows, cap, ri,
                       aff, boxes);
  else if (out_dt == kF32)
    hipLaunchKernelGGL((rrc_band_kernel<Tin, HWC, 0>), grid, dim3(kThreads), lds, st, dst, s, a, nb, pl.rows, cap, ri,
                       aff, boxes);
  else
    return -1;
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int random_resized_crop(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t batch,
                        const AugmentSpec& a, int hwc, const RowIndex& ri, const Affine& aff, int32_t* boxes_out,
                        int path, hipStream_t st) {
  if (batch <= 0) return 0;
  if (boxes_out == nullptr) return -3;  // [batch, 5] int32 device buffer: boxes are drawn there first
  if (a.channels < 1 || a.channels > kMaxAffineChannels || a.in_h < 1 || a.in_w < 1 || a.out_h < 1 || a.out_w < 1 ||
      a.out_w > 8192)  // FastDiv range: (band pixel index) * out_w < 2^32
    return -2;
  if (path < 0 || path > 2) return -2;
  switch (in_dt) {
    case kU8:
      return hwc ? launch_rrc<uint8_t, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st)
                 : launch_rrc<uint8_t, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st);
    case kF32:
      return hwc ? launch_rrc<float, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st)
                 : launch_rrc<float, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st);
    case kBF16:
      return hwc ? launch_rrc<uint16_t, 1>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st)
                 : launch_rrc<uint16_t, 0>(dst, out_dt, src, batch, a, ri, aff, boxes_out, path, st);
  }
  return -1;
}

}  // namespace ddl
