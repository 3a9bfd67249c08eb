// Host-side launchers of the ddl_amd gfx950 kernels. Every launcher enqueues on
// the given stream, never synchronises, never allocates (graph-capturable,
// guide G9) and returns 0 or a hipError_t / negative argument error.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace ddl {

// permute.hip ---------------------------------------------------------------
// dst[r, :] = cast(src[source_row(ri, r), :]) (scatter=0)
// dst[source_row(ri, r), :] = src[r, :]       (scatter=1, same dtype only)
// scatter | kHostSource: src is pinned, device-mapped host memory (a zero-copy gather): plain loads; device
// sources are gathered with non-temporal loads (they stream through once; the fresh batch stays in the MALL)
// max_blocks > 0 caps the grid (grid-stride over tiles), e.g. to keep a
// zero-copy gather out of pinned host memory on a few CUs.
constexpr int kHostSource = 2;
int gather_rows(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t n_rows, int64_t row_elems,
                const RowIndex& ri, const Affine& aff, int scatter, int64_t max_blocks, hipStream_t st);
// out[i] = feistel_perm(base + i), i < count
int feistel_indices(int64_t* out, int64_t count, int64_t base, const FeistelKeys& keys, hipStream_t st);

// collate.hip ---------------------------------------------------------------
// Image collate: src [B, H*W, C] (HWC, u8 / f32 / bf16) -> dst [B, C, H*W]
// bf16 / f32 with out = x * scale[c] + bias[c]; rows gathered through ri.
int collate_hwc_to_chw(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t batch, int64_t pixels,
                       int32_t channels, const RowIndex& ri, const Affine& aff, hipStream_t st);
// Column-group split of a [n, nValues] row batch into up to 8 contiguous
// outputs dst_k [n, width_k] (reference tuple-of-splits batches,
// ddl/mpi_dataloader.py:195-196, made contiguous), with fused gather + cast.
struct SplitSpec {
  void* dst[8];
  int32_t width[8];
  int32_t n_groups;
  int32_t out_dt;
  // split only: rows land in consecutive output slots of slot_rows rows, slot_stride bytes apart
  // (a whole window's batches in one launch); 0 = one contiguous [n_rows, width] block per group
  int64_t slot_rows;
  int64_t slot_stride;
};
int split_columns(const SplitSpec& spec, const void* src, int32_t in_dt, int64_t n_rows, int64_t n_values,
                  const RowIndex& ri, hipStream_t st);
// Inverse: spec.dst[g] are the SOURCE groups [*, width[g]] (dtype in_dt), dst is [n_rows, n_values] of
// spec.out_dt; row r of dst is row source_row(ri, r) of every group.
int pack_columns(const SplitSpec& spec, void* dst, int32_t in_dt, int64_t n_rows, int64_t n_values,
                 const RowIndex& ri, hipStream_t st);

// augment.hip ---------------------------------------------------------------
// RandomResizedCrop (+ flip, + per-channel affine, + cast) of gathered images:
// src rows [in_h, in_w, C] (hwc=1) or [C, in_h, in_w]; out [B, C, out_h, out_w].
// Crop parameters are drawn on the device from hash(seed, sample_base + source
// row) by a per-image pre-pass into boxes_out (required, [B, 5] int32 device
// buffer: y, x, h, w, flip), which the resampling kernel then reads.
struct AugmentSpec {
  uint64_t seed;
  int64_t sample_base;
  // optional [batch] crop keys (e.g. global sample ids of rows that were exchanged between ranks);
  // null: the key is sample_base + the image's source row
  const int64_t* sample_ids;
  int32_t in_h, in_w, out_h, out_w, channels;
  float scale_min, scale_max, ratio_min, ratio_max, flip_p;
};
struct CropBox {
  int32_t y, x, h, w, flip;
};
int random_resized_crop(void* dst, int32_t out_dt, const void* src, int32_t in_dt, int64_t batch,
                        const AugmentSpec& a, int hwc, const RowIndex& ri, const Affine& aff, int32_t* boxes_out,
                        int path, hipStream_t st);

// tokens.hip ----------------------------------------------------------------
// Pad: row b takes tokens[offsets[b] : offsets[b+1]] (truncated to seq_len);
// writes out_tokens [B, S] (pad_id fill), attn_mask [B, S] (u8 or null) and
// position_ids [B, S] (i32/i64 or null).
// Pack: row r holds the token span [row_start[r], row_end[r]) of the flat
// stream; seg_offsets (sorted sequence starts, n_seg+1 entries) drive the
// per-token position id (reset at every sequence start) and segment id.
struct TokenSpec {
  const void* tokens;          // int32 tokens, or uint16 when tok16 (narrow on the wire, widened here)
  const int64_t* offsets;      // pad mode: [B+1]
  const int64_t* row_start;    // pack mode: [R]
  const int64_t* row_end;      // pack mode: [R]
  const int64_t* seg_offsets;  // pack mode: [n_seg+1]
  int64_t n_seg;
  int32_t* out_tokens;
  uint8_t* attn_mask;
  void* position_ids;
  int32_t* segment_ids;        // pack mode only (or null)
  int32_t* cu_seqlens_out;     // pack mode: int32 copy of seg_offsets[0..n_seg] (varlen-attention ABI; or null)
  int64_t rows;
  int64_t seq_len;
  int32_t pad_id;
  int32_t pos_is_i64;
  int32_t mode;  // 0 pad, 1 pack
  int32_t tok16;  // 1: tokens are uint16 (vocabularies < 65536 cross PCIe at 2 B per token)
  // > rows: rows [rows, fill_rows) are written as padding (pad_id, mask 0, position 0, segment -1), so a
  // packed batch has a fixed shape [fill_rows, seq_len] (static shapes for graphs / compiled steps)
  int64_t fill_rows;
  // pack mode, plan built on the device (pack_plan_device): {n_rows, n_seg} read by the kernel instead of
  // `rows` / `n_seg`, so plan and pack are two launches with no host round trip (fill_rows = the plan's
  // row capacity; n_rows < 0, an overflowed plan, writes every row as padding)
  const int64_t* dev_counts;
};
int pad_pack_tokens(const TokenSpec& spec, hipStream_t st);

// In-order greedy packing plan of B ragged sequences, computed on the device (one workgroup): the same
// plan as the host's pack_plan (runtime/arena.cpp). Sequences longer than seq_len are split into seq_len
// segments; row r = segments [P(r), P(r + 1)) where P(r + 1) = the furthest segment end within seq_len of
// P(r)'s start. The row starts are the orbit of segment 0 under that jump, built by pointer doubling
// (orbit[2^t + i] = jump^(2^t)(orbit[i])), log2(rows) rounds instead of a rows-long dependent chain.
struct PackPlanSpec {
  const int64_t* offsets;  // [n + 1] flat token offsets of the sequences
  int64_t n;
  int64_t seq_len;
  int64_t max_segs;      // seg_offsets holds max_segs + 1 entries
  int64_t max_rows;      // row_start / row_end hold max_rows entries
  int64_t* seg_offsets;  // out: segment starts + the end
  int64_t* row_start;    // out
  int64_t* row_end;      // out
  int64_t* counts;       // out: {n_rows, n_seg}; n_rows = -1 when a capacity was exceeded
  int32_t* scratch;      // >= pack_plan_scratch_ints(max_segs, max_rows) ints (used when LDS is too small)
};
int64_t pack_plan_scratch_ints(int64_t max_segs, int64_t max_rows);
int pack_plan_device(const PackPlanSpec& spec, hipStream_t st);
// Several independent token batches (the sub-batches of one multi-batch window) in one launch per
// kMaxTokenSubs of them: grid.y = sub-batch.
constexpr int kMaxTokenSubs = 16;
int pad_pack_tokens_multi(const TokenSpec* specs, int n, hipStream_t st);

// bucket.hip ----------------------------------------------------------------
// Owner bucketing of a global batch for the resident loader's exchange: positions
// [pos0, pos0 + count) of the Feistel permutation `keys`, sample idx owned by rank
// idx / shard_rows. bucket_send writes this rank's samples (idx - lo) in position
// order (count = GB); bucket_recv maps each position of this rank's slice
// (count = LB) to its row in the all-to-all receive buffer, whose block from
// source q starts at offsets[q].
constexpr int kMaxBucketWorld = 64;
struct BucketSpec {
  FeistelKeys keys;
  int64_t pos0;
  int64_t count;
  int64_t shard_rows;
  int64_t lo;
  int32_t rank;
  int32_t world;
  int64_t offsets[kMaxBucketWorld];
};
int bucket_send(const BucketSpec& sp, int64_t* send_rows, hipStream_t st);
int bucket_recv(const BucketSpec& sp, int64_t* inv, hipStream_t st);

// misc.hip ------------------------------------------------------------------
// Sum of the 32-bit words of [ptr, ptr+bytes) added into *out (u64). Two
// stages through `scratch` (>= kChecksumMaxBlocks u64). Debug batch checksums
// and the bench consumer step.
constexpr int64_t kChecksumMaxBlocks = 1024;
// Streaming 16 B copy (bandwidth roofline probe); bytes and both pointers 16 B aligned.
int stream_copy(const void* src, void* dst, int64_t bytes, int blocks, hipStream_t st);
// One 4 B read per `page` bytes of [ptr, ptr + bytes) (e.g. a host-mapped source before zero-copy gathers);
// sink >= blocks u32 (device memory).
int touch_pages(const void* ptr, int64_t bytes, int64_t page, uint32_t* sink, int blocks, hipStream_t st);
int checksum_words(const void* ptr, int64_t bytes, uint64_t* out, uint64_t* scratch, int64_t scratch_len,
                   hipStream_t st);
// Streaming form: partials[b] += block b's share (grid = n_partials, fixed for the
// life of the accumulator); checksum_finalize adds sum(partials) into *out.
int checksum_accumulate(const void* ptr, int64_t bytes, uint64_t* partials, int64_t n_partials, hipStream_t st);
int checksum_finalize(const uint64_t* partials, int64_t n_partials, uint64_t* out, hipStream_t st);
// Per-column sum / sum of squares / min / max of an [n, cols] f32 matrix
// (reference harness normalisation stats, tests/run_ddl.py:45-77).
int column_stats(const float* src, int64_t n, int64_t cols, float* out_sum, float* out_sumsq, float* out_min,
                 float* out_max, hipStream_t st);

}  // namespace ddl
