/* Exercises the MR_* C API end to end (world size 1): every op family, the
 * multi-block reduce protocol, user hash/compare callbacks, cross-MR open/close
 * and file chunk mapping. Exits non-zero on the first failed check. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmapreduce.h"

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                      \
    }                                                               \
  } while (0)

/* ints 0..n-1, key = i % 7 (int), value = i (int64) */
static void gen(int itask, void *kv, void *app) {
  int n = *(int *)app;
  for (int i = itask; i < n; i += 4) {
    int k = i % 7;
    int64_t v = i;
    MR_kv_add(kv, (char *)&k, 4, (char *)&v, 8);
  }
}

static void gen_multi(int itask, void *kv, void *app) {
  int keys[3] = {1, 2, 3};
  int64_t vals[3] = {10, 20, 30};
  MR_kv_add_multi_static(kv, 3, (char *)keys, 4, (char *)vals, 8);
  char ks[] = "ab\0cde\0";
  int kb[2] = {3, 4};
  char vs[] = "xyz";
  int vb[2] = {1, 2};
  MR_kv_add_multi_dynamic(kv, 2, ks, kb, vs, vb);
  (void)itask; (void)app;
}

static int64_t sums[7];
static int blocks_seen = 0;

static void sum_reduce(char *key, int kb, char *mv, int nv, int *vb, void *kv, void *app) {
  int64_t s = 0;
  int total = nv;
  int nblock = 1;
  void *mr = NULL;
  if (!mv) {
    mr = (void *)vb;
    total = (int)MR_multivalue_blocks(mr, &nblock);
    blocks_seen += nblock;
  }
  int cnt = 0;
  for (int b = 0; b < nblock; ++b) {
    int n = nv;
    if (mr) n = MR_multivalue_block(mr, b, &mv, &vb);
    char *p = mv;
    for (int j = 0; j < n; ++j) {
      int64_t x;
      memcpy(&x, p, 8);
      s += x;
      p += vb[j];
      cnt++;
    }
  }
  if (cnt != total) fails++;
  sums[*(int *)key] = s;
  MR_kv_add(kv, key, kb, (char *)&s, 8);
  (void)app;
}

static int my_hash(char *key, int kb) { (void)kb; return *(int *)key; }

static int cmp_int_desc(char *a, int al, char *b, int bl) {
  (void)al; (void)bl;
  int x = *(int *)a, y = *(int *)b;
  return (x < y) - (x > y);
}

static int nscan = 0;
static void scan_kv(char *k, int kb, char *v, int vb, void *app) { nscan++; (void)k; (void)kb; (void)v; (void)vb; (void)app; }

static int last_key = 1 << 30, order_ok = 1;
static void scan_order(char *k, int kb, char *v, int vb, void *app) {
  int x = *(int *)k;
  if (x > last_key) order_ok = 0;
  last_key = x;
  (void)kb; (void)v; (void)vb; (void)app;
}

static void emit_into(uint64_t i, char *k, int kb, char *v, int vb, void *kv, void *app) {
  /* write into another (open) MR instead of our own KV */
  MR_kv_add(MR_kv_open(app), k, kb, v, vb);
  (void)i; (void)kv;
}

static uint64_t chunk_bytes = 0;
static int chunk_lines = 0;
static void chunk_map(int itask, char *str, int size, void *kv, void *app) {
  chunk_bytes += (uint64_t)size;
  for (int i = 0; i < size; ++i)
    if (str[i] == '\n') chunk_lines++;
  MR_kv_add(kv, (char *)&itask, 4, NULL, 0);
  (void)app;
}

/* keyalign / valuealign: every pointer handed to a host callback is aligned
   (reference src/keyvalue.cpp:345-352); odd-length keys make the packed
   layout misaligned, so the engine must re-lay them out */
static int misaligned = 0, aligned_seen = 0;
static void gen_odd(int itask, void *kv, void *app) {
  char k[32], v[32];
  (void)app;
  for (int i = 0; i < 300; ++i) {
    int kl = 1 + (i * 7 + itask) % 11, vl = 1 + (i * 5) % 13;
    for (int j = 0; j < kl; ++j) k[j] = (char)('a' + (i + j) % 5);
    for (int j = 0; j < vl; ++j) v[j] = (char)('0' + (i + j) % 10);
    MR_kv_add(kv, k, kl, v, vl);
  }
}
static void scan_aligned(char *k, int kb, char *v, int vb, void *app) {
  (void)kb; (void)vb; (void)app;
  aligned_seen++;
  if (((uintptr_t)k % 8) || ((uintptr_t)v % 16)) misaligned++;
}
static void reduce_aligned(char *k, int kb, char *mv, int nv, int *vb, void *kv, void *app) {
  (void)kb; (void)nv; (void)vb; (void)kv; (void)app;
  aligned_seen++;
  if (((uintptr_t)k % 8) || ((uintptr_t)mv % 16)) misaligned++;
}

int main(int argc, char **argv) {
  const char *tmpdir = argc > 1 ? argv[1] : ".";
  MR_set_error_mode(1);
  void *mr = MR_create(MR_comm_world());
  CHECK(MR_num_procs(mr) == 1 && MR_my_proc(mr) == 0);
  int n = 100000;
  CHECK(MR_map(mr, 4, gen, &n) == (uint64_t)n);
  CHECK(MR_map_add(mr, 1, gen_multi, NULL, 1) == (uint64_t)n + 5);

  /* drop the mixed-layout pairs again: rebuild only the int keys */
  void *ints = MR_create(NULL);
  CHECK(MR_map(ints, 4, gen, &n) == (uint64_t)n);
  CHECK(MR_aggregate(ints, my_hash) == (uint64_t)n);
  CHECK(MR_convert(ints) == 7);
  MR_set_memsize(ints, -4096); /* 4 KB pages: every key goes through the multi-block path */
  CHECK(MR_reduce(ints, sum_reduce, NULL) == 7);
  CHECK(blocks_seen > 7);
  for (int k = 0; k < 7; ++k) {
    int64_t want = 0;
    for (int i = k; i < n; i += 7) want += i;
    CHECK(sums[k] == want);
  }

  /* built-in device reducers */
  void *c = MR_create(NULL);
  MR_set_chunk_bytes(c, 4096); /* MI355X settings: tiny shuffle rounds, pipelined collate */
  MR_set_pipeline(c, 1);
  MR_set_hbm_budget(c, 0);
  MR_map(c, 4, gen, &n);
  CHECK(MR_collate(c, NULL) == 7);
  CHECK(MR_reduce_builtin(c, "count", "int32") == 7);
  CHECK(MR_kv_stats(c, 0) == 7);

  /* compress (local combiner) + sort with a user compare */
  void *s = MR_copy(ints);
  CHECK(MR_sort_keys(s, cmp_int_desc) == 7);
  MR_scan_kv(s, scan_order, NULL);
  CHECK(order_ok);
  CHECK(MR_sort_keys_flag(s, 1) == 7);
  nscan = 0;
  CHECK(MR_scan_kv(s, scan_kv, NULL) == 7 && nscan == 7);

  void *cm = MR_create(NULL);
  MR_map(cm, 4, gen, &n);
  blocks_seen = 0;
  CHECK(MR_compress(cm, sum_reduce, NULL) == 7);

  /* clone / collapse / scrunch */
  void *cl = MR_create(NULL);
  MR_map(cl, 4, gen, &n);
  CHECK(MR_clone(cl) == (uint64_t)n);
  void *co = MR_create(NULL);
  MR_map(co, 4, gen, &n);
  char key[] = "all";
  CHECK(MR_collapse(co, key, 4) == 1);
  void *sc = MR_create(NULL);
  MR_map(sc, 4, gen, &n);
  CHECK(MR_scrunch(sc, 1, key, 4) == 1);

  /* sort_multivalues flag and compare forms */
  void *sm = MR_create(NULL);
  MR_map(sm, 4, gen, &n);
  MR_convert(sm);
  CHECK(MR_sort_multivalues_flag(sm, -2) == 7);

  /* cross-MR writes through open/close (reference luby_find/sssp pattern) */
  void *dst = MR_create(NULL);
  MR_open(dst);
  void *srcmr = MR_create(NULL);
  MR_map(srcmr, 4, gen, &n);
  void *sink = MR_create(NULL);
  CHECK(MR_map_mr(sink, srcmr, emit_into, dst) == 0);
  CHECK(MR_close(dst) == (uint64_t)n);
  MR_destroy(sink);

  /* add / broadcast / gather on one rank */
  CHECK(MR_add(dst, srcmr) == 2 * (uint64_t)n);
  CHECK(MR_broadcast(dst, 0) == 2 * (uint64_t)n);
  CHECK(MR_gather(dst, 1) == 2 * (uint64_t)n);

  /* file chunks split at newlines */
  char path[4096];
  snprintf(path, sizeof(path), "%s/capi_lines.txt", tmpdir);
  FILE *f = fopen(path, "w");
  for (int i = 0; i < 5000; ++i) fprintf(f, "line %d of the chunked file\n", i);
  fclose(f);
  char *files[1] = {path};
  void *fc = MR_create(NULL);
  CHECK(MR_map_file_char(fc, 7, 1, files, 0, 0, '\n', 80, chunk_map, NULL) == 7);
  CHECK(chunk_lines == 5000);

  /* print to a file */
  snprintf(path, sizeof(path), "%s/capi_print.txt", tmpdir);
  MR_print_file(c, path, 0, -1, 1, 1, 1);
  f = fopen(path, "r");
  int lines = 0;
  char buf[256];
  while (f && fgets(buf, sizeof buf, f)) lines++;
  if (f) fclose(f);
  CHECK(lines == 7);

  /* alignment of callback pointers */
  void *al = MR_create(NULL);
  MR_set_keyalign(al, 8);
  MR_set_valuealign(al, 16);
  CHECK(MR_map(al, 2, gen_odd, NULL) == 600);
  MR_scan_kv(al, scan_aligned, NULL);
  CHECK(aligned_seen == 600 && misaligned == 0);
  MR_collate(al, NULL);
  aligned_seen = 0;
  MR_reduce(al, reduce_aligned, NULL);
  CHECK(aligned_seen > 10 && misaligned == 0);
  MR_set_keyalign(al, 3);
  MR_map(al, 1, gen_odd, NULL);
  CHECK(MR_scan_kv(al, scan_aligned, NULL) == 0 && strstr(MR_last_error(), "alignment") != NULL);
  MR_destroy(al);

  /* errors come back as codes in error mode 1 */
  void *e = MR_create(NULL);
  CHECK(MR_convert(e) == 0 && strlen(MR_last_error()) > 0);

  void *all[] = {mr, ints, c, s, cm, cl, co, sc, sm, dst, srcmr, fc, e};
  for (unsigned i = 0; i < sizeof(all) / sizeof(all[0]); ++i) MR_destroy(all[i]);
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("ALL OK\n");
  return 0;
}
