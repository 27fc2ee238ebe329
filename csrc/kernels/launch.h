// Host-side launcher declarations for the hand-written CDNA4 (gfx950) kernels.
//
// Every launcher takes raw device pointers plus the HIP stream to run on; the
// engine layer (csrc/engine/*.cpp) owns allocation through the ATen caching
// allocator and always passes the current torch stream, so kernels, RCCL
// collectives (issued by c10d on its own stream with event fences) and torch
// ops are correctly ordered.
//
// The kernels replace the CPU hot loops of MR-MPI
// and the CUDA/Thrust InvertedIndex map (K1-K5, /root/reference/cuda/InvertedIndex.cu:79-135,324-370).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace mrh {
namespace k {

// ---------------------------------------------------------------- scan.hip
// Exclusive prefix sum. `out` has n+1 entries: out[n] = total. in/out may not alias.
// temp must hold scan_temp_bytes(n) bytes.
size_t scan_temp_bytes(int64_t n);
void exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, void* temp, hipStream_t s);
void exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t s);
// lengths (int32) -> int64 offsets (n+1)
void lengths_to_offsets(const int32_t* len, int64_t* off, int64_t n, void* temp, hipStream_t s);

// ---------------------------------------------------------------- radix.hip
// Stable LSD radix sort of (uint64 key, uint32 value) pairs over digits
// [begin_bit, end_bit), one one-sweep (decoupled look-back) kernel per 8-bit
// pass. skip_trivial: passes whose digit is constant over all keys are
// skipped using the up-front global histogram (one host sync); false = no
// host sync at all. Result ends in keys_out/vals_out.
// temp must hold radix_temp_bytes(n) bytes. All buffers have n entries.
size_t radix_temp_bytes(int64_t n);
void radix_sort_u64_u32(const uint64_t* keys_in, const uint32_t* vals_in, uint64_t* keys_out,
                        uint32_t* vals_out, uint64_t* keys_alt, uint32_t* vals_alt, int64_t n,
                        int begin_bit, int end_bit, void* temp, hipStream_t s,
                        int* passes_run = nullptr, bool skip_trivial = true);

// ---------------------------------------------------------------- hash.hip
// lookup3 hashlittle(key, len, seed) (bit-exact with Bob Jenkins' reference) per key.
void hash32_fixed(const uint8_t* kdata, int kw, int64_t n, uint32_t seed, uint32_t* out, hipStream_t s);
void hash32_var(const uint8_t* kdata, const int64_t* koff, int64_t n, uint32_t seed, uint32_t* out,
                hipStream_t s);
// 64-bit grouping hash (lookup3 hashlittle2: c<<32|b)
void hash64_fixed(const uint8_t* kdata, int kw, int64_t n, uint64_t* out, hipStream_t s);
void hash64_var(const uint8_t* kdata, const int64_t* koff, int64_t n, uint64_t* out, hipStream_t s);
// destination rank = h % P, plus per-destination pair counts (atomic, LDS-aggregated)
void partition_dest(const uint32_t* h, int64_t n, int P, int32_t* dest, int64_t* counts, hipStream_t s);

// ---------------------------------------------------------------- shuffle.hip
// Pairs per partition tile (block): nb = ceil(n / part_tile()) blocks.
int part_tile();
// owner per pair (dest_in given, or hashlittle(key, kb, P) % P written to
// dest_out) and per-(owner d, block b) tables at [d*nb + b]: pair counts, and
// key / value byte sums for variable columns (koff / voff non-null; kbytes /
// vbytes null otherwise)
void part_count(const int32_t* dest_in, const uint8_t* kd, int kw, const int64_t* koff, const int64_t* voff,
                int64_t n, int P, int nb, int32_t* dest_out, int64_t* cnt, int64_t* kbytes, int64_t* vbytes,
                hipStream_t s);
// stable scatter into owner buckets: cbase = exclusive scan of cnt. Fixed
// columns (kw / vw >= 0) are copied into ksend / vsend; for variable columns
// perm (send position -> input pair) and klen / vlen are written instead
void part_scatter(const int32_t* dest, int64_t n, int P, int nb, const int64_t* cbase, const uint8_t* kd, int kw,
                  const uint8_t* vd, int vw, const int64_t* koff, const int64_t* voff, uint8_t* ksend,
                  uint8_t* vsend, int64_t* perm, int32_t* klen, int32_t* vlen, hipStream_t s);
// variable rows gathered by an int64 permutation into dst at doff
void copy_var_i64(const uint8_t* src, const int64_t* soff, const int64_t* perm, int64_t n, uint8_t* dst,
                  const int64_t* doff, hipStream_t s);
// this rank's exchange header row (3P + 2 int64) from the scanned tables
void part_header(const int64_t* cs, const int64_t* ks, const int64_t* vs, int P, int nb, int kw, int vw,
                 int64_t kcode, int64_t vcode, int64_t* hdr, hipStream_t s);
// counts[v % P] (counts zeroed by the caller) of non-negative int64 ids
void count_mod(const int64_t* v, int64_t n, int P, int64_t* counts, hipStream_t s);
// byte sizes [P][R] of the R pieces of each bucket of a variable column
void piece_bytes(const int64_t* soff, const int64_t* start, int P, int R, int64_t* out, hipStream_t s);

// ---------------------------------------------------------------- segops.hip
// marks[seg[s]] += 1 for s in [1, nseg) with seg[s] < nval (marks zeroed
// here, nval entries): inclusive scan -> segment id per value
void seg_marks(const int64_t* seg, int64_t nseg, int64_t nval, int64_t* marks, hipStream_t s);
// counts[idx[i]]++ over K bins (zeroed here), global atomics
void histogram(const int64_t* idx, int64_t n, int64_t K, int64_t* counts, hipStream_t s);
// f[i] = v[i] != 0 ; out[pos[i]] = i for non-zero v (pos = exclusive scan of f)
void nz_flags(const uint64_t* v, int64_t n, int32_t* f, hipStream_t s);
void compact_nz(const uint64_t* v, const int64_t* pos, int64_t n, int64_t* out, hipStream_t s);
// bool-mask compaction: f[i] = m[i] != 0 (int64); out[pos[i]] = i for set m[i] (pos = exclusive scan of f)
void mask_flags(const uint8_t* m, int64_t n, int64_t* f, hipStream_t s);
void compact_mask(const uint8_t* m, const int64_t* pos, int64_t n, int64_t* out, hipStream_t s);
// idx[j] = index of q[j] in sorted unique keys[0, n), or -1 (binary search per query)
void lookup_sorted(const int64_t* keys, int64_t n, const int64_t* q, int64_t m, int64_t* idx, hipStream_t s);

// ---------------------------------------------------------------- kvops.hip
// Sort-key construction: fixed-width keys (kw<=8) loaded little-endian into a
// uint64 and transformed so that unsigned order == requested order.
// mode: 0 raw unsigned LE, 1 int32, 2 uint64, 3 float, 4 double, 7 int64, 8 uint32
// descending: bitwise NOT after transform. Also writes iota into idx.
void make_sortkeys_fixed(const uint8_t* data, int w, int64_t n, int mode, bool descending,
                         uint64_t* keys, uint32_t* idx, hipStream_t s);
// String keys (flag 5/6): big-endian 8-byte prefix starting at byte `start` of each
// key (zero padded); descending inverts.
void make_sortkeys_strprefix(const uint8_t* data, const int64_t* off, int64_t n, int64_t start,
                             bool descending, uint64_t* keys, uint32_t* idx, hipStream_t s);
void iota_u32(uint32_t* idx, int64_t n, hipStream_t s);
// device tie-break rounds of the string sort (kvops.hip; engine.cpp sort_perm_column)
void str_groups(const uint64_t* ks, const uint8_t* alive, const uint32_t* head_in, int64_t n, bool desc,
                uint32_t* head_out, hipStream_t s);
void str_active(const uint64_t* ks, const uint8_t* alive, const uint32_t* head, int64_t n, bool desc, uint32_t* active,
                hipStream_t s);
void str_refine(const uint32_t* active, const uint32_t* pos, const uint32_t* gid_incl, const uint32_t* perm,
                const uint8_t* data, const int64_t* off, int64_t n, int64_t start, bool desc, int32_t* where,
                uint64_t* nk, uint64_t* gk, hipStream_t s);
void str_apply(const uint32_t* order, const int32_t* where, const uint64_t* nk, int64_t m, const uint32_t* perm_in,
               uint32_t* perm_out, uint64_t* ks, uint8_t* alive, hipStream_t s);
// rows of width w gathered by idx
void gather_fixed(const uint8_t* src, int w, const uint32_t* idx, int64_t n, uint8_t* dst, hipStream_t s);
void gather_fixed_i64idx(const uint8_t* src, int w, const int64_t* idx, int64_t n, uint8_t* dst,
                         hipStream_t s);
// variable rows: step 1 lengths in gathered order; step 2 copy bytes (dst_off already scanned)
void gather_var_lengths(const int64_t* src_off, const uint32_t* idx, int64_t n, int32_t* len,
                        hipStream_t s);
void gather_var_copy(const uint8_t* src, const int64_t* src_off, const uint32_t* idx, int64_t n,
                     uint8_t* dst, const int64_t* dst_off, hipStream_t s);
// sorted u64 keys -> head flags (uint32 0/1)
void head_flags_u64(const uint64_t* keys, int64_t n, uint32_t* flags, hipStream_t s);
// head positions: seg[pos[i]] = i where flags[i]; seg[nseg] = n  (pos = exclusive scan of flags)
void compact_heads(const uint32_t* flags, const uint32_t* pos, int64_t n, int64_t* seg, hipStream_t s);
// exact narrow keys: fixed keys of nw (<= 8) 8-byte words -> out[i] = OR of
// word w << s[w] (s[w] < 0: the word is zero in every key), idx[i] = i
struct PackShifts {
  int nw;
  int s[8];
};
void pack_words(const uint64_t* kd, int64_t n, const PackShifts& sh, uint64_t* out, uint32_t* idx, hipStream_t s);
// out[i] = vd[i] | OR of key word w << s[w] (narrow keys and values on one u64)
void pack_kv(const uint64_t* kd, const uint64_t* vd, int64_t n, const PackShifts& sh, uint64_t* out, hipStream_t s);
// narrow pairs past one u64 (kvops.hip k_pack_kv_split): out[i] =
// rest << vbits | value, bkt[i] = the bucket (bkt may be null when B == 0);
// hi >= 0: ordered cut (bucket K >> hi, rest the low hi bits), hi < 0: mixed
// cut (rest K >> B, bucket low B bits ^ mix(rest)); vw 4 or 8; shifts s[w]
// place key word w in K
void pack_kv_split(const uint64_t* kd, const void* vd, int vw, int64_t n, const PackShifts& sh, int vbits, int B, int hi,
                   uint64_t* out, int32_t* bkt, hipStream_t s);
// keys[j * nw + w] from the sorted heads (rest) of bucket `bucket` (the same
// B, hi as the packing); bits.s[w]: significant bits of word w
void unpack_split(const uint64_t* heads, int64_t m, int bucket, int B, int hi, const PackShifts& sh,
                  const PackShifts& bits, uint64_t* keys, hipStream_t s);
// vout[i] = words[i] & (2^vbits - 1) as u32 (vw 4) or u64 (vw 8)
void split_values(const uint64_t* words, int64_t n, int vbits, int vw, void* vout, hipStream_t s);
// segments of sorted packed words (kvops.hip k_seg_packed_*): per-tile head
// counts, then (tbase = their exclusive scan) segment starts, head key bits
// ((w >> vb) & km) and values (w & (2^vb - 1), vw 4 or 8)
int64_t seg_packed_tiles(int64_t n);
void seg_packed_count(const uint64_t* w, int64_t n, int vb, uint64_t km, int64_t* tcnt, hipStream_t s);
void seg_packed_write(const uint64_t* w, int64_t n, int vb, uint64_t km, const int64_t* tbase, int64_t* seg,
                      uint64_t* heads, void* vout, int vw, hipStream_t s);
// head bitmap H (nw 64-bit words): cnt[w] = popcount; then seg[pos[w] + k] =
// position of the k-th set bit of word w, seg[pos[nw]] = n
void bits_count(const uint64_t* H, int64_t nw, uint32_t* cnt, hipStream_t s);
void bits_compact(const uint64_t* H, int64_t nw, const uint32_t* pos, int64_t n, int64_t* seg, hipStream_t s);
// after grouping by 64-bit hash: count elements whose key bytes differ from their group head
void verify_groups_var(const uint8_t* kdata, const int64_t* koff, const uint32_t* perm,
                       const uint32_t* flags, const uint32_t* pos, const int64_t* seg, int64_t n,
                       unsigned long long* mismatches, hipStream_t s);
void verify_groups_fixed(const uint8_t* kdata, int kw, const uint32_t* perm, const uint32_t* flags,
                         const uint32_t* pos, const int64_t* seg, int64_t n,
                         unsigned long long* mismatches, hipStream_t s);
// per-destination byte totals of variable rows (for alltoallv byte splits)
void dest_byte_counts(const int32_t* dest, const int64_t* off, int64_t n, int P, int64_t* bytes,
                      hipStream_t s);
// offsets -> int32 lengths
void offsets_to_lengths(const int64_t* off, int64_t n, int32_t* len, hipStream_t s);

// ---------------------------------------------------------------- segreduce.hip
// Segmented reductions over KMV values (seg has nseg+1 entries).
// op: 0 sum, 1 min, 2 max ; dtype: 0 int32, 1 int64, 2 float32, 3 float64
void seg_reduce(const void* vals, int dtype, int op, const int64_t* seg, int64_t nseg, int64_t nval, void* out,
                hipStream_t s);
void seg_count(const int64_t* seg, int64_t nseg, int32_t* out, hipStream_t s);

// ---------------------------------------------------------------- text.hip
// InvertedIndex map: find every `<a href="` in text[0,n) and emit the URL that
// follows (up to the next '"' or end of text). Two passes: count, then emit.
// Block tile = 4 KiB of text.
int64_t url_num_tiles(int64_t n);
void url_count(const uint8_t* text, int64_t n, uint32_t* tile_counts, hipStream_t s);
// tile_off = exclusive scan of tile_counts (n_tiles+1)
void url_emit_starts(const uint8_t* text, int64_t n, const uint32_t* tile_off, int64_t* starts,
                     hipStream_t s);
// per url: length (excl. terminator) -> key length incl. NUL
void url_lengths(const uint8_t* text, int64_t n, const int64_t* starts, int64_t nurl,
                 int32_t* keylen, hipStream_t s);
void url_copy(const uint8_t* text, const int64_t* starts, const int64_t* koff, int64_t nurl,
              uint8_t* kdata, hipStream_t s);
// whitespace tokenizer (wordfreq): word starts/lengths; keys are word + NUL
int64_t tok_num_tiles(int64_t n);
// wordfreq pairs in one pass (text.hip k_tok_count2 / k_tok_emit2): per tile
// the words and the key bytes (non-separators + one NUL per word), then the
// key bytes and key offsets written from their exclusive scans (toff_w u32,
// toff_b i64; koff[nw] is the caller's)
void tok_count2(const uint8_t* text, int64_t n, uint32_t* tile_words, uint32_t* tile_bytes, hipStream_t s);
void tok_emit2(const uint8_t* text, int64_t n, const uint32_t* toff_w, const int64_t* toff_b, int64_t* koff,
               uint8_t* kd, hipStream_t s);
void tok_count(const uint8_t* text, int64_t n, uint32_t* tile_counts, hipStream_t s);
void tok_emit(const uint8_t* text, int64_t n, const uint32_t* tile_off, int64_t* starts,
              int32_t* keylen, hipStream_t s);
// copy `n` strings text[starts[i] .. +len-1] into kdata at koff[i], then NUL
void copy_strings_nul(const uint8_t* text, const int64_t* starts, const int64_t* koff, int64_t n,
                      uint8_t* kdata, hipStream_t s);
void fill_i32(int32_t* p, int64_t n, int32_t v, hipStream_t s);
// out[i] = number of sorted (unsigned) splitters < keys[i] (right: <= keys[i],
// numpy searchsorted side='right'); nsplit <= 4096
void bucket_by_splitters(const uint64_t* keys, int64_t n, const uint64_t* split, int nsplit, int32_t* out,
                         hipStream_t s, bool right = false);

// ---------------------------------------------------------------- graph.hip
// R-MAT edges: counter-based Philox RNG; edge e of stream `seed` is a pure
// function of (seed, e). Writes (vi, vj) uint64 pairs.
void rmat_edges(uint64_t* edges, int64_t nedges, int nlevels, float a, float b, float c, float d,
                float fraction, uint64_t seed, uint64_t first_edge, hipStream_t s);

// ---------------------------------------------------------------- graphops.hip
size_t pr_scratch_bytes(int64_t nval);
void pr_contrib(const int64_t* seg, int64_t nseg, int64_t nedge, const int32_t* src, const float* w, const float* r,
                float* out, void* scratch, hipStream_t s);
void pr_combine(const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const float* recv,
                const int32_t* vid, float* grp, float* acc, void* scratch, hipStream_t s);
void scatter_f32(const float* v, const int32_t* idx, int64_t n, float* out, hipStream_t s);
int pr_update_blocks(int64_t n);
// PageRank plan build (graphops.hip): source-sorted packed edges -> run
// degrees, degree relabel, packed (destination group << 32 | new source)
// edge keys and their unpack
void pr_pack_src(const int64_t* e, int64_t n, int P, bool swap, uint64_t* out, hipStream_t s);
void pr_heads(const uint64_t* sorted, int64_t n, uint32_t* flags, hipStream_t s);
void pr_run_degree(const uint64_t* sorted, const int64_t* seg, int64_t nrun, uint32_t* deg, hipStream_t s);
void pr_degkey(const uint32_t* deg, int64_t n, uint64_t* key, uint32_t* iota, hipStream_t s);
void pr_relabel(const uint32_t* order, const uint32_t* deg, int64_t n, int32_t* nid, int64_t* order64,
                uint8_t* dangling, float* invdeg, unsigned long long* ndangling, int32_t* degn, hipStream_t s);
// out[k] = in[min(k * stride, n - 1)] for k < ns
void sample_i64(const int64_t* in, int64_t n, int64_t stride, int64_t ns, int64_t* out, hipStream_t s);
// rb (nullable, nr + 1 entries): hot source ranges [rb[r], rb[r+1]), ids >=
// rb[nr] form range nr; the range goes above the dbits destination bits
void pr_pack(const uint64_t* su, int64_t n, int P, int64_t nlmax, bool local, bool swapped, const int32_t* nid,
             const int32_t* rb, int nr, int dbits, uint64_t* out, hipStream_t s);
// multi-GPU plan (owner of v = sigma(v) % P, vmix.h; mix false: sigma = id):
// edges -> (sigma(v) << 32 | sigma(u)) + source owner; (sv << 32 | su) ->
// (sv << 32 | su / P) in place; (sv << 32 | lu) -> (sv << 32 | base +
// nid[lu]) + destination owner; at the destination owner (sv << 32 |
// pos) -> ((range << dbits | nid[sv / P]) << 32 | pos), the range of the
// interleaved source id (pos % S) * P + pos / S; owned global ids
// sigma^-1(order * P + me)
void pr_mix_pack(const int64_t* e, int64_t n, int P, int64_t N, bool mix, uint64_t* out, int32_t* dest, hipStream_t s);
void pr_localize(uint64_t* p, int64_t n, int P, hipStream_t s);
void pr_pack_dst(const uint64_t* su, int64_t n, int P, int64_t base, const int32_t* nid, uint64_t* out, int32_t* dest,
                 hipStream_t s);
void pr_pack_gather(const uint64_t* in, int64_t n, int P, int64_t S, const int32_t* nid, const int32_t* rb, int nr,
                    int dbits, uint64_t* out, hipStream_t s);
void pr_unmix_ids(const int64_t* order, int64_t n, int P, int me, int64_t N, bool mix, int64_t* ids, hipStream_t s);
void pr_unpack(const uint64_t* sorted, int64_t n, int32_t* src, uint32_t* flags, hipStream_t s);
// deg[v] += out-edges of v; e sorted on the source (low word) bits >= shift
// (shift <= 10), deg zeroed by the caller
void pr_deg_window(const uint64_t* e, int64_t m, int shift, uint32_t* deg, hipStream_t s);
// the same with the heads as a bitmap H (ws_words(n) u32, zeroed by the caller)
void pr_unpack_bits(const uint64_t* sorted, int64_t n, int32_t* src, uint32_t* H, hipStream_t s);
void pr_group_hi(const uint64_t* sorted, const int64_t* seg, int64_t ngrp, int64_t* hi, hipStream_t s);
void pr_group_vid(const int64_t* hi, int64_t ngrp, const int32_t* nid, int64_t dmask, int32_t* vid, hipStream_t s);
// XCD source ranges: destinations per combine tile (log2); first group of
// every (range, tile) (R * (ntile + 1) int64); the tiled partial-sum combine
int pr_tile_bits();
void pr_range_offsets(const int64_t* hi, int64_t ngrp, int dbits, int R, int64_t ntile, int64_t* off, hipStream_t s);
// one step's combine + update per tile of destinations (new ids): partial
// sums -> r_new, c = r_new / outdeg, per-tile (L1 delta, dangling mass)
// partials (2 * ntile doubles)
// stats[0], stats[1] = sums of the tile step's (L1 delta, dangling mass) partials
void pr_partials_sum(const double* part, int64_t ntile, double* stats, hipStream_t s);
void pr_tile_step(const float* send, const int32_t* ghi, const int64_t* off, int R, int64_t ntile, int64_t ndst,
                  const float* r, float* rn, const uint8_t* dangling, float base, float alpha, const double* dmass,
                  double invN, const float* invdeg, float* cout, double* partial, hipStream_t s);
void pr_update(float* acc, const float* r, float* rn, const uint8_t* dangling, int64_t n, float base,
               float alpha, const double* dmass, double invN, const float* invdeg, float* cout, double* partial,
               hipStream_t s);

// generic edge-plan propagation (cc_find / sssp / luby_find); dtype 1 int64, 2 float, 3 double;
// op 0 sum, 1 min, 2 max; w may be null (else value = x[src] + w)
size_t plan_scratch_bytes(int64_t n);
void plan_gather_reduce(int dtype, const int64_t* seg, int64_t nseg, int64_t ne, const int32_t* src, const void* x,
                        const void* w, int op, void* out, void* scratch, hipStream_t s);
void plan_combine(int dtype, const int64_t* seg, int64_t ngrp, int64_t nrecv, const int32_t* perm, const void* recv,
                  const int32_t* vid, int op, void* grp, void* acc, void* scratch, hipStream_t s);
// static-segment index (wavesegred.h) for plans whose segments never change:
// head bitmap H (ws_words(nval) u32) + per-wave segment base (ws_waves(nval) i64)
int64_t ws_words(int64_t nval);
int64_t ws_waves(int64_t nval);
void ws_index(const int64_t* seg, int64_t nseg, int64_t nval, uint32_t* H, int64_t* wbase, hipStream_t s);
// the per-wave segment bases only (H built elsewhere, e.g. pr_unpack_bits)
void ws_bases(const int64_t* seg, int64_t nseg, int64_t nval, int64_t* wbase, hipStream_t s);
// out[s] = OP_{e in seg s} x[src[e]] (+ w[e]); dtype/op as plan_gather_reduce;
// scratch: ws_scratch_bytes(nval)
size_t ws_scratch_bytes(int64_t nval);
// sched (nullable): 8 x slen wave ids (-1 = none); blocks b and b + 8 share an
// XCD, so slot b % 8 runs the waves of row b % 8 (an XCD-pinned schedule)
// nx: entries of x (> 0 enables the hot-prefix kernel: x[0, 32k) in LDS,
// wavesegred.h k_ws_gather_reduce_hot; MRH_PR_HOT=<ids> / 0)
void ws_gather_reduce(int dtype, const uint32_t* H, const int64_t* wbase, int64_t nval, const int32_t* src,
                      const void* x, const void* w, int op, void* out, void* scratch, hipStream_t s,
                      const int32_t* sched = nullptr, int64_t slen = 0, int64_t nx = 0);
// tri_find wedges: all pairs of each neighbour group with d >= 2 (gidx:
// those groups, wscan: the exclusive scan of their C(d,2), ngw + 1 entries);
// wedge ids [w0, w0 + nwedge), output slot i holds wedge w0 + i, so a huge
// group set is generated in bounded chunks; tg: scratch of
// wedge_tiles(nwedge) + 1 entries (each tile's first group)
int64_t wedge_tiles(int64_t nwedge);
void wedges(const int64_t* seg, const int64_t* gidx, const int64_t* wscan, int64_t ngw, const int64_t* nb,
            const int64_t* centre, int64_t w0, int64_t nwedge, int64_t* out_edge, int64_t* out_centre, int64_t* tg,
            hipStream_t s);
// the same wedges in the compact layout: out_key = min << vb | max, out_centre u32
void wedges_compact(const int64_t* seg, const int64_t* gidx, const int64_t* wscan, int64_t ngw, const int64_t* nb,
                    const int64_t* centre, int64_t w0, int64_t nwedge, int vb, int64_t* out_key, uint32_t* out_centre,
                    int64_t* tg, hipStream_t s);

// ---------------------------------------------------------------- pbpr.hip
// propagation-blocked PageRank (graphplan.cpp PageRankPlan, one GPU)
int pb_bin_size();  // destinations per bin (16-bit offsets)
// vals[out_pos[j]] = c[src[j]] over the phase-1 order
void pb_phase1(const int32_t* src, const int32_t* out_pos, int64_t m, const float* c, float* vals, hipStream_t s);
// per unit (bin, [e0, e1)): LDS sums of vals by 16-bit destination -> acc
void pb_phase2(const float* vals, const uint16_t* dst, const int32_t* ub, const int64_t* ue0, const int64_t* ue1,
               const uint8_t* uex, int64_t nunit, int64_t nv, float* acc, hipStream_t s);
// out_pos[perm2[k]] = k ; dst2[k] = dst1[perm2[k]] & (bin - 1)
void pb_layout(const int32_t* perm2, const int32_t* dst1, int64_t m, int32_t* out_pos, uint16_t* dst2, hipStream_t s);

// ---------------------------------------------------------------- tri.hip
// triangle enumeration on a degree-oriented CSR (packed u64 edges lo<<32|hi)
// [n, 2] int64 edges -> packed min << 32 | max (self loops -> 0, ids outside
// [0, nvert) set *bad); col = low
// words of the oriented keys; rank[perm[r]] = r
void tri_pack(const int64_t* e, int64_t n, int64_t nvert, uint64_t* out, unsigned int* bad, hipStream_t s);
void tri_col(const uint64_t* okeys, int64_t m, uint32_t* col, hipStream_t s);
void tri_rank(const int32_t* perm, int64_t n, int32_t* rank, hipStream_t s);
void tri_degree(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s);
// partitioned degree count (tri.hip): buckets of 2^tri_deg_bucket_bits()
// vertices (-1: too many buckets, use tri_degree); lo runs; bucket counts;
// scatter of the high endpoints as u16 into their buckets; per-(bucket,
// piece) LDS histograms added to deg (plain stores where whole != 0)
int tri_deg_buckets(int64_t nvert);
// deg[low word of e[i]] += 1 with one global atomic per element (the fallback
// of the partitioned count for more than 2^27 bins)
void count_low_atomic(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s);
int tri_deg_bucket_bits();
void tri_deg_lo(const uint64_t* e, int64_t m, uint32_t* deg, hipStream_t s);
void tri_deg_count(const uint64_t* e, int64_t m, int nb, unsigned int* bcount, hipStream_t s);
void tri_deg_scatter(const uint64_t* e, int64_t m, int nb, unsigned long long* cursor, uint16_t* out, hipStream_t s);
void tri_deg_hist(const uint16_t* ids, const unsigned long long* bstart, const uint64_t* items, const uint32_t* ilen,
                  const uint8_t* whole, int64_t nitems, int64_t nvert, uint32_t* deg, hipStream_t s);
// packed (a,b) -> rank ids (min<<32|max) with rank = (degree, id) order
void tri_orient(const uint64_t* e, int64_t m, const uint32_t* rank, uint64_t* out, hipStream_t s);
// per oriented edge in [e0,e1): cnt (nullable) and atomic total
void tri_count(const int64_t* rowptr, const uint32_t* col, const uint64_t* okeys, int64_t e0, int64_t e1,
               uint32_t* cnt, unsigned long long* total, hipStream_t s);
// vertex-centric LDS-hash count over vertices [u0,u1); big: scratch u32[2*(u1-u0)], nbig: zeroed u32[2]
// H/hb/K: hub bitmaps built by tri_hub_count (H null: none) — probes of a hub
// neighbour test bits of its row instead of walking its adjacency list
void tri_count_hash(const int64_t* rowptr, const uint32_t* col, int64_t u0, int64_t u1, uint32_t* big,
                    uint32_t* nbig, unsigned long long* total, hipStream_t s, const uint64_t* H = nullptr,
                    int64_t hb = 0, int64_t K = 0);
// triangles whose lowest vertex is a hub (rank >= hb = nvert - K) among the
// vertices [u0, u1), by AND/popcount of hub adjacency bitmaps; H: scratch of
// K * K / 8 bytes (K a multiple of 64, <= 524288)
// hub rows grouped by the middle vertex v (tri.hip "pull"): prep packs the
// hub edges [ea, ea + n) as (v - hb) << 32 | (e - ea) and the end of every
// edge's source row; after the keys-only sort (tks) and tptr (first item of
// every v, K + 1), npieces -> exclusive scan off (K + 1) -> tri_hub_pull
void tri_hub_pull_prep(const uint32_t* col, const uint64_t* okeys, const int64_t* rowptr, int64_t hb, int64_t ea,
                       int64_t n, uint64_t* tk, uint32_t* endx, hipStream_t s);
void tri_hub_pull_npieces(const int64_t* tptr, const int64_t* rowptr, int64_t hb, int64_t K, int64_t* np,
                          hipStream_t s);
int64_t tri_hub_pull_max_items(int64_t n, int64_t K);
void tri_hub_pull(const int64_t* rowptr, const uint32_t* col, int64_t hb, int64_t K, int64_t ea, const uint64_t* tks,
                  const int64_t* tptr, const uint32_t* endx, const int64_t* off, uint64_t* items, uint64_t* big,
                  unsigned int* nbig, const uint64_t* H, unsigned long long* total, hipStream_t s);
void tri_hub_count(const int64_t* rowptr, const uint32_t* col, int64_t hb, int64_t K, int64_t u0, int64_t u1,
                   uint64_t* H, unsigned long long* total, hipStream_t s);
// ---------------------------------------------------------------- ccmr.hip
// cc_find_mr callbacks (oink/cc_find.cpp:119-330); zone keys carry the hot
// bit 63 and the salting rank at pshift. Emitting steps take pos = exclusive
// scan of their flags (ccmr_len_flags / _winner_flags / _hot_flags).
void ccmr_len_flags(const int64_t* voff, int64_t nval, int64_t w, int64_t* f, hipStream_t s);
void ccmr_edge_zone_of(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                       int64_t* zone_of, hipStream_t s);
void ccmr_edge_zone_emit(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                         const int64_t* zone_of, const int64_t* pos, int64_t* edge, int64_t* zone, hipStream_t s);
void ccmr_winner_flags(const int64_t* seg, int64_t nkey, const int64_t* z, int64_t nval, int64_t* f, hipStream_t s);
void ccmr_winner_emit(const int64_t* seg, int64_t nkey, const int64_t* z, int64_t nval, const int64_t* pos,
                      int64_t* big, int64_t* pad, hipStream_t s);
void ccmr_invert(const int64_t* v, const int64_t* zn, int64_t n, int P, int pshift, uint64_t seed, int64_t* key,
                 int64_t* val, hipStream_t s);
void ccmr_hot_flags(const int64_t* zn, int64_t n, int64_t* f, hipStream_t s);
void ccmr_zone_multi(const int64_t* zn, const int64_t* pad, int64_t n, int P, int pshift, const int64_t* pos,
                     int64_t* key, int64_t* val, hipStream_t s);
void ccmr_reassign_seg(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                       int64_t lmask, int64_t nthresh, int64_t* zone_out, hipStream_t s);
void ccmr_reassign_emit(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
                        const int64_t* zone_seg, const int64_t* pos, int64_t* v, int64_t* zone, hipStream_t s);

// ---------------------------------------------------------------- graphmr.hip
// sssp_mr (oink/sssp.cpp:244-360) and luby_find_mr (oink/luby_find.cpp:120-344)
// callbacks; voff may be null for fixed-width values of vw bytes where noted
void sssp_pick(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const uint8_t* vd, int64_t* out,
               int64_t* changed, hipStream_t s);
void sssp_pick_emit(const int64_t* keys, int64_t nkey, const int64_t* dist, const int64_t* pos, int64_t* okey,
                    int64_t* odist, hipStream_t s);
// best = ~0 and idx = ~0 and found = 0 on entry
void sssp_best(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vd, int64_t nval,
               unsigned long long* best, unsigned long long* idx, int64_t* found, hipStream_t s);
void sssp_relax_flags(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                      int64_t nval, const unsigned long long* idx, const int64_t* found, int64_t* fe, int64_t* fp,
                      hipStream_t s);
void sssp_relax_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, const uint8_t* vd,
                     int64_t nval, const unsigned long long* idx, const int64_t* found, const int64_t* pe,
                     const int64_t* pp, int64_t* ekey, int64_t* eval, int64_t* pkey, int64_t* pval, hipStream_t s);
void luby_nonloop(const int64_t* e, int64_t n, int64_t* f, hipStream_t s);
void luby_random(const int64_t* e, int64_t n, int64_t seed, const int64_t* pos, int64_t* out, hipStream_t s);
// mark = 0 on entry; mode 0 flag-0 VFLAG, 1 value > 16 B, 2 value == 16 B, 3 value > 0 B
void luby_mark(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const uint8_t* vd, int64_t nval,
               int mode, int64_t* mark, hipStream_t s);
void luby_key_flags(const int64_t* mark, int64_t nkey, int64_t want, int64_t* f, hipStream_t s);
void luby_edge_emit(const int64_t* keys, int64_t nkey, const int64_t* pos, int64_t* okey, int64_t* oval,
                    hipStream_t s);
// mark null: f = value length != 16
void luby_value_flags(const int64_t* seg, int64_t nkey, const int64_t* voff, int64_t vw, const int64_t* mark,
                      int64_t nval, int64_t want, int64_t* f, hipStream_t s);
void luby_vert_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, int64_t vw,
                    const uint8_t* vd, int64_t nval, const int64_t* p24, int64_t* k24, int64_t* v24, int64_t* k16,
                    int64_t* v16, hipStream_t s);
void luby_edges_emit(const int64_t* seg, int64_t nkey, const int64_t* keys, const int64_t* voff, int64_t vw,
                     const uint8_t* vd, int64_t nval, const int64_t* pf, int64_t* kf, int64_t* kn, hipStream_t s);
void luby_mis_emit(const int64_t* keys, int64_t nkey, const int64_t* pos, int64_t* out, hipStream_t s);

// ---------------------------------------------------------------- trimr.hip
// tri_find_mr callbacks (oink/tri_find.cpp:104-325); edge rows are int64
// pairs, degree rows int32 pairs
void trimr_first_degree(const int64_t* seg, int64_t nkey, const int64_t* key, const int64_t* nbr, int64_t nval,
                        int64_t* edge, int32_t* deg, hipStream_t s);
void trimr_second_degree(const int64_t* seg, int64_t nkey, const int32_t* v, int64_t nval, int32_t* out,
                         hipStream_t s);
void trimr_low_degree(const int64_t* e, const int32_t* dg, int64_t n, int64_t* key, int64_t* val, hipStream_t s);
// fixed 8-byte values (marker: the key's first vertex), value-parallel in tiles: phase 0 sets
// marked[key] (zeroed by the caller) for the keys holding a marker, phase 1
// writes each tile's count of centres of marked keys to tcount[tile], phase 2
// writes rows (centre, edge key) from tbase[tile] on. compact_vb > 0: keys are
// one packed word vi << vb | vj and values u32 (else EDGE keys, int64 values)
// tk (trimr_emit_tiles(nval) + 1 entries, from trimr_emit_tile_keys): the key
// of every tile's first value, found once for the three phases
int64_t trimr_emit_tiles(int64_t nval);
void trimr_emit_tile_keys(const int64_t* seg, int64_t nkey, int64_t nval, int64_t* tk, hipStream_t s);
void trimr_emit_fixed(int phase, const int64_t* seg, int64_t nkey, int64_t nval, const void* vals, uint8_t* marked,
                      int64_t* tcount, const int64_t* tbase, const int64_t* ekey, int64_t* out, int compact_vb,
                      const int64_t* tk, hipStream_t s);
// cnt[s] = wedge centres of edge segment s if it holds the edge marker, else 0
// (voff: variable-width values, the marker is empty; voff null: fixed 8-byte
// values vals, the marker is the key's first vertex)
void trimr_emit_count(const int64_t* seg, int64_t nkey, const int64_t* voff, const int64_t* vals, const int64_t* ekey,
                      int64_t* cnt, hipStream_t s);
// rows (centre, e0, e1) at pos[s].. (pos = exclusive scan of cnt)
void trimr_emit_write(const int64_t* seg, int64_t nkey, const int64_t* voff, const uint8_t* vdata,
                      const int64_t* ekey, const int64_t* pos, int64_t* out, hipStream_t s);

// dense 0/1 int8 adjacency of the top T ranks (cb = nvert - T), T x T, zeroed here
void tri_core_build(const int64_t* rowptr, const uint32_t* col, int64_t cb, int64_t T, int8_t* A, hipStream_t s);
// CSR row pointers of sorted oriented keys
void tri_rowptr(const uint64_t* okeys, int64_t m, int64_t nvert, int64_t* rowptr, hipStream_t s);
// triangles (u,v,w) as 3 u64 at off[e-e0] (off: exclusive scan of cnt, n+1 entries)
void tri_emit(const int64_t* rowptr, const uint32_t* col, const uint64_t* okeys, int64_t e0, int64_t e1,
              const int64_t* off, uint64_t* out, hipStream_t s);

// ---------------------------------------------------------------- apps.hip
// InvertedIndex output formatting: "key\tname name ... \n" per KMV key.
void ii_value_len(const int32_t* vals, int64_t nval, const int64_t* name_off, int32_t* lenv, hipStream_t s);
void ii_key_len(const int64_t* koff, int64_t nseg, int32_t* lens, hipStream_t s);
void ii_write(const uint8_t* kd, const int64_t* koff, const int32_t* vals, int64_t nval, const int64_t* seg,
              int64_t nseg, const int64_t* cv, const int64_t* cs, const uint8_t* names, const int64_t* name_off,
              uint8_t* out, hipStream_t s);

}  // namespace k
}  // namespace mrh

// ---------------------------------------------------------------- group.hip
// exact hash-dictionary group-by (HashDict / GroupIndex, csrc/engine/grouper.h)
namespace mrh {
namespace k {
// one slot of the table (32 bytes; all zero = empty)
struct alignas(32) DictSlot {
  unsigned long long hash;  // key hash (a zero hash is stored as 1), 0 = empty
  int32_t gid1;             // group id + 1, 0 until published
  int32_t len;              // key bytes
  uint32_t key[4];          // the key's first 16 bytes, zero padded
};
struct DictTable {
  DictSlot* slots;            // [cap]
  uint64_t mask;              // cap - 1 (cap a power of two)
  int64_t* rep;               // [cap] first row of a group, -1 until published
  uint64_t* ghash;            // [cap] hash of a group
  unsigned long long* ctr;    // [groups, collisions, rows left unassigned, full flag]
  int64_t limit;              // no new group past this many
};
// group every row row0+i (i < n) of the key column (kd, koff | kw): gid[row]
// = its group or -1 when the table was full; h: optional
// precomputed hashes (else lookup3 hashlittle2 of the bytes); retry: only
// rows whose gid is -1.
void dict_insert(const uint8_t* kd, const int64_t* koff, int kw, const uint64_t* h, int64_t n, int64_t row0,
                 const DictTable& t, int32_t* gid, bool retry, hipStream_t s);
void dict_rehash(const DictSlot* old_slots, int64_t old_cap, DictSlot* new_slots, int64_t new_cap, hipStream_t s);
// out[j] = hash of row j*n/m, j < m
void dict_sample(const uint8_t* kd, const int64_t* koff, int kw, int64_t n, int64_t m, uint64_t* out, hipStream_t s);
// cnt[g] = rows with gid == g, g < m (LDS histograms, no per-row global atomic)
// ws: dict_counts_ws_elems() u32 of scratch
void dict_counts(const int32_t* gid, int64_t n, int64_t m, uint64_t* cnt, uint32_t* ws, hipStream_t s);
int64_t dict_counts_ws_elems();
// cnt[j] = gcount[order[j]]
void dict_ranked_counts(const uint32_t* order, int64_t m, const uint64_t* gcount, int64_t* cnt, hipStream_t s);
// aoff[i] = poff[i] + base for i in [0, n]
void grp_append_off(const int64_t* poff, int64_t n, int64_t base, int64_t* aoff, hipStream_t s);
// rank[order[j]] = j, heads[j] = rep[order[j]]
void grp_rank(const uint32_t* order, int64_t m, const int64_t* rep, uint32_t* rank, uint32_t* heads, hipStream_t s);
// key[i] = rank[gid[i]]
void grp_pairkey(const int32_t* gid, int64_t n, const uint32_t* rank, uint64_t* key, hipStream_t s);
// CSR segments of dense sorted ranks 0..m-1
void grp_seg(const uint64_t* sorted_rank, int64_t n, int64_t m, int64_t* seg, hipStream_t s);
}  // namespace k
}  // namespace mrh

// ---------------------------------------------------------------- wordcount.hip
// In-mapper combining word count (see wordcount.hip). slots/counts: table of
// `cap` (power of two) entries; ctr[0] used slots, ctr[1] arena bytes;
// newlist receives the slots claimed by this chunk (>= words-in-chunk entries).
namespace mrh {
namespace k {
void wc_count(const uint8_t* text, int64_t n, uint64_t* slots, uint32_t* counts, int64_t cap, int32_t* newlist,
              uint64_t* ctr, uint64_t used0, const uint8_t* arena, hipStream_t s);
void wc_migrate(const uint8_t* text, int64_t n, uint64_t* slots, int64_t cap, int32_t* newlist, uint64_t* ctr,
                uint64_t used0, uint8_t* arena, int64_t max_new, hipStream_t s);
void wc_rehash(const uint64_t* old_slots, const uint32_t* old_counts, int64_t old_cap, const uint8_t* arena,
               uint64_t* new_slots, uint32_t* new_counts, int64_t new_cap, hipStream_t s);
void wc_keys(const uint64_t* slots, const int64_t* idx, int64_t nk, const uint8_t* arena, int64_t* starts,
             int32_t* lens, hipStream_t s);
}  // namespace k
}  // namespace mrh

// ---------------------------------------------------------------- kmeans.hip
namespace mrh {
namespace k {
bool kmeans_supported(int D, int K);
// acc[K*(D+1)] (fp64, zeroed by the caller) += per-cluster coordinate sums and counts
void kmeans_assign_accumulate(const float* pts, int64_t n, int D, const float* cen, int K, double* acc,
                              hipStream_t s);
// acc[K*(D+1)] += coordinate sums and counts of points already assigned (idx[n] in [0, K))
void kmeans_accumulate(const float* pts, int64_t n, int D, const int64_t* idx, int K, double* acc, hipStream_t s);
}  // namespace k
}  // namespace mrh

// ---------------------------------------------------------------- util.hip
// Engine primitives in place of ATen expressions on hot paths (one launch or
// two each, on the caller's stream, no host sync). The reductions need
// minmax_scratch_words(rows, cols) int64 words of device scratch.
namespace mrh {
namespace k {
// pieces of pinned host memory (device-accessible) gathered into one device
// buffer by a kernel (zero-copy reads over PCIe): one launch instead of one
// copy-engine command per piece (tools/h2d_pieces_bench.hip: 40 x 1.6 MB
// pieces at 55.8 GB/s vs 41.6 GB/s by one hipMemcpyAsync each)
struct PieceTable {
  static constexpr int kMax = 48;
  const uint8_t* src[kMax];
  int64_t dst_off[kMax];
  int64_t bytes[kMax];
  int n = 0;
};
void gather_pieces(const PieceTable& t, uint8_t* dst, hipStream_t s);
int64_t minmax_scratch_words(int64_t rows, int cols);
// per column of a row-major [rows, cols] int64 matrix (cols <= 8): out[c] =
// min, out[cols + c] = max (rows == 0: LLONG_MAX / LLONG_MIN)
void col_minmax_i64(const int64_t* p, int64_t rows, int cols, int64_t* scratch, int64_t* out, hipStream_t s);
// out[0] = min, out[1] = max of int32 values (widened)
void minmax_i32(const int32_t* p, int64_t n, int64_t* scratch, int64_t* out, hipStream_t s);
void fill_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
// dst[i] = src[i] + v (dst may be src)
void add_i64(const int64_t* src, int64_t* dst, int64_t n, int64_t v, hipStream_t s);
// out[i] = ((h[i] >> shift) & mask) % M
void part_of_hash(const uint64_t* h, int64_t n, int shift, uint64_t mask, int M, int32_t* out, hipStream_t s);
// edges [n, 2]: out[0] = min over both ends, out[1] = 1 if some a >= b, out[2] = max
void edge_probe(const int64_t* e, int64_t n, int64_t* scratch, int64_t* out, hipStream_t s);
// keys = [a; b], values = [b; a] (2n each)
void edge_both_ways(const int64_t* e, int64_t n, int64_t* key, int64_t* val, hipStream_t s);
// key = a << vb | b, value = (int32) a
void edge_pack(const int64_t* e, int64_t n, int vb, uint64_t* key, int32_t* val, hipStream_t s);
// value = a
void edge_first(const int64_t* e, int64_t n, int64_t* val, hipStream_t s);
// edge_upper (reference oink map_edge_upper): flag[i] = a != b; then the
// flagged rows as (min, max) at pos[i] (the exclusive scan of the flags)
void edge_ne_flags(const int64_t* e, int64_t n, uint32_t* flag, hipStream_t s);
void edge_upper_write(const int64_t* e, int64_t n, const uint32_t* pos, int64_t* out, hipStream_t s);
}  // namespace k
}  // namespace mrh
