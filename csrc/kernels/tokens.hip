// Variable-length token collate (BASELINE config 4:
// seq_len = 4096 token sequences, on-device pad/pack).
//
// Pad mode: B ragged sequences -> [B, S] tokens padded with pad_id, a u8
// attention mask and position ids, truncated to S.
// Tokens arrive as int32, or as uint16 (tok16: vocabularies below 65536 ship 2 B per token over PCIe and
// are widened to int32 here, in the same pass).
// Pack mode: consecutive sequences are packed into rows of S tokens (plan
// computed on the host: row r = flat token span [row_start, row_end)); the
// position id restarts at every sequence boundary and a segment id marks
// which sequence a token belongs to (what varlen attention consumes).
//
// Grid: one workgroup per (row, chunk of kSpan positions), so a 64 x 4096
// batch is 512 workgroups (the first form ran one workgroup per row: 64 of the
// 256 CUs busy). Each lane writes 4 consecutive positions as 16 B (tokens,
// i32 ids) / 4 B (mask) vectors. Pack mode copies the sequence starts into
// LDS once per workgroup (one coalesced read) and binary-searches there; the
// first form binary-searched global memory for every token, a chain of
// ~log2(n_seg) dependent loads per position.
#include "common.h"
#include "launch.h"

namespace ddl {
namespace {

constexpr int kThreads = 128;
constexpr int kSpan = kThreads * 4;  // positions per workgroup
constexpr int kSegCap = 1024;        // sequence starts staged in LDS (8 KB)

// index of the last entry <= v of the sorted a[0..n) (a[0] <= v)
template <typename At>
__device__ __forceinline__ int64_t last_le(At at, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (at(mid) <= v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo - 1;
}

template <typename At>
__device__ __forceinline__ void emit4(const TokenSpec& sp, int64_t row, int64_t p0, int64_t start, int64_t len,
                                      At seg_at) {
  const int64_t S = sp.seq_len;
  const int32_t* src = static_cast<const int32_t*>(sp.tokens) + start;
  const uint16_t* src16 = static_cast<const uint16_t*>(sp.tokens) + start;
  int32_t tok[4], pos[4], seg[4];
  uint8_t msk[4];
  int64_t s = -1;  // current sequence (pack mode): searched once, then advanced
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t p = p0 + k;
    const bool valid = p < len;
    tok[k] = valid ? (sp.tok16 ? static_cast<int32_t>(src16[p]) : src[p]) : sp.pad_id;
    msk[k] = valid ? 1 : 0;
    if (sp.mode == 0) {
      pos[k] = valid ? static_cast<int32_t>(p) : 0;
      seg[k] = 0;
    } else if (valid) {
      const int64_t g = start + p;  // flat token index
      if (s < 0)
        s = last_le(seg_at, sp.n_seg + 1, g);
      else
        while (s + 1 <= sp.n_seg && seg_at(s + 1) <= g) ++s;
      pos[k] = static_cast<int32_t>(g - seg_at(s));
      seg[k] = static_cast<int32_t>(s);
    } else {
      pos[k] = 0;
      seg[k] = -1;
    }
  }
  const int64_t o = row * S + p0;
  if (p0 + 4 <= S && (S % 4 == 0)) {
    *reinterpret_cast<int4*>(sp.out_tokens + o) = make_int4(tok[0], tok[1], tok[2], tok[3]);
    if (sp.attn_mask) {
      const uint32_t m = msk[0] | (msk[1] << 8) | (msk[2] << 16) | (static_cast<uint32_t>(msk[3]) << 24);
      *reinterpret_cast<uint32_t*>(sp.attn_mask + o) = m;
    }
    if (sp.position_ids) {
      if (sp.pos_is_i64) {
        int64_t* pp = static_cast<int64_t*>(sp.position_ids) + o;
        *reinterpret_cast<longlong2*>(pp) = make_longlong2(pos[0], pos[1]);
        *reinterpret_cast<longlong2*>(pp + 2) = make_longlong2(pos[2], pos[3]);
      } else {
        *reinterpret_cast<int4*>(static_cast<int32_t*>(sp.position_ids) + o) = make_int4(pos[0], pos[1], pos[2], pos[3]);
      }
    }
    if (sp.segment_ids) *reinterpret_cast<int4*>(sp.segment_ids + o) = make_int4(seg[0], seg[1], seg[2], seg[3]);
  } else {
    for (int k = 0; k < 4 && p0 + k < S; ++k) {
      sp.out_tokens[o + k] = tok[k];
      if (sp.attn_mask) sp.attn_mask[o + k] = msk[k];
      if (sp.position_ids) {
        if (sp.pos_is_i64)
          static_cast<int64_t*>(sp.position_ids)[o + k] = pos[k];
        else
          static_cast<int32_t*>(sp.position_ids)[o + k] = pos[k];
      }
      if (sp.segment_ids) sp.segment_ids[o + k] = seg[k];
    }
  }
}

// One workgroup = (row, chunk) `bx` of batch `sp`. Blocks past the batch's rows (a multi-batch launch is
// sized for its largest sub-batch) only do block 0's cu_seqlens copy; the exit is block-uniform.
__device__ __forceinline__ void pad_pack_block(const TokenSpec& spec, uint32_t bx, int32_t chunks, int64_t* seg_lds) {
  TokenSpec sp = spec;
  if (sp.dev_counts != nullptr) {  // plan built on the device: its row / segment counts (block-uniform loads)
    sp.rows = sp.dev_counts[0] < 0 ? 0 : sp.dev_counts[0];
    sp.n_seg = sp.dev_counts[0] < 0 ? 0 : sp.dev_counts[1];
  }
  const uint32_t row = bx / static_cast<uint32_t>(chunks);
  const bool live = row < (sp.fill_rows > sp.rows ? sp.fill_rows : sp.rows);  // data row or padding row
  const int64_t p0 = static_cast<int64_t>(bx - row * static_cast<uint32_t>(chunks)) * kSpan +
                     static_cast<int64_t>(threadIdx.x) * 4;
  int64_t start = 0, len = 0;  // a padding row: len 0, every position written as padding
  if (row < sp.rows) {
    if (sp.mode == 0) {
      start = sp.offsets[row];
      len = sp.offsets[row + 1] - start;
    } else {
      start = sp.row_start[row];
      len = sp.row_end[row] - start;
    }
  }
  if (len > sp.seq_len) len = sp.seq_len;
  if (len < 0) len = 0;
  const bool staged = sp.mode == 1 && sp.n_seg + 1 <= kSegCap;  // batch-uniform
  if (staged && live)
    for (int64_t i = threadIdx.x; i <= sp.n_seg; i += kThreads) seg_lds[i] = sp.seg_offsets[i];
  if (sp.cu_seqlens_out != nullptr && bx == 0)  // owned copy of the sequence starts (cu_seqlens)
    for (int64_t i = threadIdx.x; i <= sp.n_seg; i += kThreads)
      sp.cu_seqlens_out[i] = static_cast<int32_t>(sp.seg_offsets[i]);
  __syncthreads();
  if (!live || p0 >= sp.seq_len) return;
  if (staged)
    emit4(sp, row, p0, start, len, [&](int64_t i) { return seg_lds[i]; });
  else
    emit4(sp, row, p0, start, len, [&](int64_t i) { return sp.seg_offsets[i]; });
}

__global__ void __launch_bounds__(kThreads) pad_pack_kernel(TokenSpec sp, int32_t chunks) {
  __shared__ int64_t seg_lds[kSegCap];
  pad_pack_block(sp, blockIdx.x, chunks, seg_lds);
}

struct TokenMulti {
  TokenSpec sub[kMaxTokenSubs];
};

__global__ void __launch_bounds__(kThreads) pad_pack_multi_kernel(TokenMulti m, int32_t chunks) {
  __shared__ int64_t seg_lds[kSegCap];
  pad_pack_block(m.sub[blockIdx.y], blockIdx.x, chunks, seg_lds);
}

// ---- device packing plan (one workgroup) ----------------------------------------------------------------
constexpr int kPlanThreads = 1024;
constexpr int kPlanWaves = kPlanThreads / 64;
constexpr int64_t kPlanLdsInts = 12288;  // 48 KB of LDS for the jump tables + the orbit, else global scratch

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t u = __shfl_up(v, d, 64);
    if (lane >= d) v += u;
  }
  return v;
}

__global__ void __launch_bounds__(kPlanThreads) pack_plan_kernel(PackPlanSpec sp) {
  __shared__ int64_t wave_tot[kPlanWaves];
  __shared__ int64_t carry_s;
  __shared__ int32_t lds[kPlanLdsInts];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int64_t S = sp.seq_len;
  if (t == 0) carry_s = 0;
  __syncthreads();
  // 1. segments: c_i = ceil(len_i / S) per sequence, exclusive scan over the sequences in 1024-wide tiles
  for (int64_t b = 0; b < sp.n; b += kPlanThreads) {
    const int64_t i = b + t;
    int64_t s0 = 0, len = 0;
    if (i < sp.n) {
      s0 = sp.offsets[i];
      len = sp.offsets[i + 1] - s0;
    }
    const int64_t c = len > 0 ? (len + S - 1) / S : 0;
    const int64_t incl = wave_incl_scan(c);
    if (lane == 63) wave_tot[wv] = incl;
    __syncthreads();
    int64_t before = carry_s;
    for (int k = 0; k < wv; ++k) before += wave_tot[k];
    const int64_t first = before + incl - c;
    for (int64_t j = 0; j < c; ++j)
      if (first + j < sp.max_segs) sp.seg_offsets[first + j] = s0 + j * S;
    __syncthreads();
    if (t == kPlanThreads - 1) carry_s = before + incl;
    __syncthreads();
  }
  const int64_t n_seg = carry_s;
  if (n_seg > sp.max_segs) {  // block-uniform exit
    if (t == 0) {
      sp.counts[0] = -1;
      sp.counts[1] = n_seg;
    }
    return;
  }
  if (t == 0) sp.seg_offsets[n_seg] = n_seg > 0 ? sp.offsets[sp.n] : 0;
  __syncthreads();
  // 2. jump tables (ping-pong) and the orbit: LDS when they fit, else the caller's scratch
  const int64_t need = 2 * (n_seg + 1) + sp.max_rows + 1;
  int32_t* base = need <= kPlanLdsInts ? lds : sp.scratch;
  int32_t* J = base;
  int32_t* J2 = base + (n_seg + 1);
  int32_t* P = base + 2 * (n_seg + 1);
  const int64_t cap = sp.max_rows + 1;  // orbit entries: the rows' starts + the terminal n_seg
  for (int64_t k = t; k <= n_seg; k += kPlanThreads) {
    int32_t m = static_cast<int32_t>(n_seg);
    if (k < n_seg) {  // furthest segment end m within S tokens of segment k's start (every segment >= 1 token)
      const int64_t lim = sp.seg_offsets[k] + S;
      int64_t lo = k + 1, hi = n_seg - k > S ? k + S : n_seg;  // seg_offsets[lo] <= lim always
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (sp.seg_offsets[mid] <= lim)
          lo = mid;
        else
          hi = mid - 1;
      }
      m = static_cast<int32_t>(lo);
    }
    J[k] = m;
  }
  if (t == 0) P[0] = 0;
  __syncthreads();
  int64_t len = 1;
  while (P[len - 1] < n_seg && len < cap) {  // P[0..len) known, J = jump^len: P[len + i] = J[P[i]]
    const int64_t add = len < cap - len ? len : cap - len;
    for (int64_t i = t; i < add; i += kPlanThreads) P[len + i] = J[P[i]];
    for (int64_t k = t; k <= n_seg; k += kPlanThreads) J2[k] = J[J[k]];
    __syncthreads();
    int32_t* tmp = J;
    J = J2;
    J2 = tmp;
    len += add;
  }
  if (P[len - 1] < n_seg) {  // more rows than max_rows (block-uniform)
    if (t == 0) {
      sp.counts[0] = -1;
      sp.counts[1] = n_seg;
    }
    return;
  }
  // 3. rows: the orbit entries before the terminal one (P strictly increases until it reaches n_seg)
  for (int64_t i = t; i < len; i += kPlanThreads) {
    if (P[i] < n_seg) {
      sp.row_start[i] = sp.seg_offsets[P[i]];
      sp.row_end[i] = sp.seg_offsets[P[i + 1]];
      if (P[i + 1] == n_seg) {
        sp.counts[0] = i + 1;
        sp.counts[1] = n_seg;
      }
    }
  }
  if (t == 0 && n_seg == 0) {
    sp.counts[0] = 0;
    sp.counts[1] = 0;
  }
}

}  // namespace

int64_t pack_plan_scratch_ints(int64_t max_segs, int64_t max_rows) { return 2 * (max_segs + 1) + max_rows + 1; }

int pack_plan_device(const PackPlanSpec& spec, hipStream_t st) {
  if (spec.seq_len <= 0 || spec.n < 0 || spec.max_segs < 0 || spec.max_rows < 0) return -2;
  if (!spec.offsets || !spec.seg_offsets || !spec.row_start || !spec.row_end || !spec.counts || !spec.scratch)
    return -2;
  if (spec.max_segs >= (int64_t{1} << 31) - 1) return -4;  // int32 segment ids in the jump tables
  hipLaunchKernelGGL(pack_plan_kernel, dim3(1), dim3(kPlanThreads), 0, st, spec);
  return static_cast<int>(hipGetLastError());
}

int pad_pack_tokens(const TokenSpec& spec, hipStream_t st) {
  const int64_t rows = spec.fill_rows > spec.rows ? spec.fill_rows : spec.rows;
  if (rows <= 0 || spec.seq_len <= 0) return 0;
  if (spec.mode == 0 && !spec.offsets) return -2;
  if (spec.mode == 1 && (!spec.row_start || !spec.row_end || !spec.seg_offsets)) return -2;
  const int64_t chunks = (spec.seq_len + kSpan - 1) / kSpan;
  if (rows * chunks >= (int64_t{1} << 31)) return -4;
  hipLaunchKernelGGL(pad_pack_kernel, dim3(static_cast<uint32_t>(rows * chunks)), dim3(kThreads), 0, st, spec,
                     static_cast<int32_t>(chunks));
  return static_cast<int>(hipGetLastError());
}

int pad_pack_tokens_multi(const TokenSpec* specs, int n, hipStream_t st) {
  for (int g = 0; g < n; g += kMaxTokenSubs) {
    TokenMulti m{};
    const int cnt = n - g < kMaxTokenSubs ? n - g : kMaxTokenSubs;
    int64_t max_rows = 1, seq_len = 0;  // >= 1 block per sub-batch: block 0 writes its cu_seqlens
    for (int j = 0; j < cnt; ++j) {
      const TokenSpec& sp = specs[g + j];
      if (sp.seq_len <= 0 || (sp.mode == 0 && !sp.offsets) ||
          (sp.mode == 1 && (!sp.row_start || !sp.row_end || !sp.seg_offsets)))
        return -2;
      if (j > 0 && sp.seq_len != seq_len) return -2;  // one chunking for the launch
      seq_len = sp.seq_len;
      if (sp.rows > max_rows) max_rows = sp.rows;
      if (sp.fill_rows > max_rows) max_rows = sp.fill_rows;
      m.sub[j] = sp;
    }
    const int64_t chunks = (seq_len + kSpan - 1) / kSpan;
    if (max_rows * chunks >= (int64_t{1} << 31)) return -4;
    hipLaunchKernelGGL(pad_pack_multi_kernel, dim3(static_cast<uint32_t>(max_rows * chunks), static_cast<uint32_t>(cnt)),
                       dim3(kThreads), 0, st, m, static_cast<int32_t>(chunks));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
  }
  return 0;
}

}  // namespace ddl
