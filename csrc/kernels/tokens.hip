// Variable-length token collate (BASELINE config 4:
// seq_len = 4096 token sequences, on-device pad/pack).
//
// Pad mode: B ragged sequences -> [B, S] tokens padded with pad_id, a u8
// attention mask and position ids, truncated to S.
// Pack mode: consecutive sequences are packed into rows of S tokens (plan
// computed on the host: row r = flat token span [row_start, row_end)); the
// position id restarts at every sequence boundary and a segment id marks
// which sequence a token belongs to (what varlen attention consumes).
//
// One workgroup per output row; each lane writes 4 consecutive positions so
// the three outputs are stored as 16 B (tokens, i32 ids) / 4 B (mask) vectors.
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ int64_t upper_bound_i64(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(kThreads) pad_pack_kernel(TokenSpec sp) {
  const int64_t row = blockIdx.x;
  const int64_t S = sp.seq_len;
  int64_t start, len;
  if (sp.mode == 0) {
    start = sp.offsets[row];
    len = sp.offsets[row + 1] - start;
  } else {
    start = sp.row_start[row];
    len = sp.row_end[row] - start;
  }
  if (len > S) len = S;
  if (len < 0) len = 0;
  int32_t* out_tok = sp.out_tokens + row * S;
  const int32_t* src = sp.tokens + start;
  for (int64_t p0 = static_cast<int64_t>(threadIdx.x) * 4; p0 < S; p0 += kThreads * 4) {
    int32_t tok[4];
    int32_t pos[4];
    int32_t seg[4];
    uint8_t msk[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t p = p0 + k;
      const bool valid = p < len;
      tok[k] = valid ? src[p] : sp.pad_id;
      msk[k] = valid ? 1 : 0;
      if (sp.mode == 0) {
        pos[k] = valid ? static_cast<int32_t>(p) : 0;
        seg[k] = 0;
      } else if (valid) {
        const int64_t g = start + p;  // flat token index
        const int64_t s = upper_bound_i64(sp.seg_offsets, sp.n_seg + 1, g) - 1;
        pos[k] = static_cast<int32_t>(g - sp.seg_offsets[s]);
        seg[k] = static_cast<int32_t>(s);
      } else {
        pos[k] = 0;
        seg[k] = -1;
      }
    }
    const bool full = (p0 + 4 <= S);
    if (full && (S % 4 == 0)) {
      *reinterpret_cast<int4*>(out_tok + p0) = make_int4(tok[0], tok[1], tok[2], tok[3]);
      if (sp.attn_mask) {
        const uint32_t m = msk[0] | (msk[1] << 8) | (msk[2] << 16) | (static_cast<uint32_t>(msk[3]) << 24);
        *reinterpret_cast<uint32_t*>(sp.attn_mask + row * S + p0) = m;
      }
      if (sp.position_ids) {
        if (sp.pos_is_i64) {
          int64_t* pp = static_cast<int64_t*>(sp.position_ids) + row * S + p0;
          *reinterpret_cast<longlong2*>(pp) = make_longlong2(pos[0], pos[1]);
          *reinterpret_cast<longlong2*>(pp + 2) = make_longlong2(pos[2], pos[3]);
        } else {
          *reinterpret_cast<int4*>(static_cast<int32_t*>(sp.position_ids) + row * S + p0) =
              make_int4(pos[0], pos[1], pos[2], pos[3]);
        }
      }
      if (sp.segment_ids)
        *reinterpret_cast<int4*>(sp.segment_ids + row * S + p0) = make_int4(seg[0], seg[1], seg[2], seg[3]);
    } else {
      for (int k = 0; k < 4 && p0 + k < S; ++k) {
        const int64_t o = row * S + p0 + k;
        out_tok[p0 + k] = tok[k];
        if (sp.attn_mask) sp.attn_mask[o] = msk[k];
        if (sp.position_ids) {
          if (sp.pos_is_i64)
            static_cast<int64_t*>(sp.position_ids)[o] = pos[k];
          else
            static_cast<int32_t*>(sp.position_ids)[o] = pos[k];
        }
        if (sp.segment_ids) sp.segment_ids[o] = seg[k];
      }
    }
  }
}

}  // namespace

int pad_pack_tokens(const TokenSpec& spec, hipStream_t st) {
  if (spec.rows <= 0 || spec.seq_len <= 0) return 0;
  if (spec.mode == 0 && !spec.offsets) return -2;
  if (spec.mode == 1 && (!spec.row_start || !spec.row_end || !spec.seg_offsets)) return -2;
  hipLaunchKernelGGL(pad_pack_kernel, dim3(static_cast<uint32_t>(spec.rows)), dim3(kThreads), 0, st, spec);
  return static_cast<int>(hipGetLastError());
}

}  // namespace ddl
