/* Word frequency through the MR_* C API of gpu_mapreduce_amd.
 *
 * Same job as the reference's examples/cwordfreq.c (C-API wordfreq with a
 * top-N listing): map every file into (word, NULL) pairs, collate, count,
 * sort by count (descending), keep each rank's top N, gather to rank 0 and
 * print the global top N.
 *
 *   cc cwordfreq.c -I../../csrc/capi -L../../gpu_mapreduce_amd -lmrhip \
 *      -Wl,-rpath,$PWD/../../gpu_mapreduce_amd -o cwordfreq
 *   ./cwordfreq [-n NTOP] file1 dir2 ...
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmapreduce.h"

static const char *WS = " \t\n\f\r";

/* map: one task per file; every whitespace-separated word becomes a key */
static void read_words(int itask, char *fname, void *kv, void *app) {
  FILE *f = fopen(fname, "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", fname);
    exit(1);
  }
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *text = (char *)malloc((size_t)n + 1);
  size_t got = fread(text, 1, (size_t)n, f);
  text[got] = '\0';
  fclose(f);
  char *save = NULL;
  for (char *w = strtok_r(text, WS, &save); w; w = strtok_r(NULL, WS, &save))
    MR_kv_add(kv, w, (int)strlen(w) + 1, NULL, 0);
  free(text);
  (void)itask;
  (void)app;
}

/* reduce: (word, [NULL...]) -> (word, int count); multi-block aware */
static void count(char *key, int kb, char *mv, int nv, int *vb, void *kv, void *app) {
  int total = nv;
  if (mv == NULL) { /* values of this key span several blocks */
    int nblock = 0;
    total = (int)MR_multivalue_blocks((void *)vb, &nblock);
  }
  MR_kv_add(kv, key, kb, (char *)&total, (int)sizeof(int));
  (void)app;
}

struct Top {
  int limit, seen;
};

/* map over the sorted MR: keep the first `limit` pairs */
static void keep_top(uint64_t i, char *key, int kb, char *val, int vb, void *kv, void *app) {
  struct Top *t = (struct Top *)app;
  if (t->seen++ < t->limit) MR_kv_add(kv, key, kb, val, vb);
  (void)i;
}

static void print_top(char *key, int kb, char *val, int vb, void *app) {
  int *left = (int *)app;
  if ((*left)-- > 0) printf("%d %s\n", *(int *)val, key);
  (void)kb;
  (void)vb;
}

int main(int argc, char **argv) {
  int ntop = 10, first = 1;
  if (argc > 2 && strcmp(argv[1], "-n") == 0) {
    ntop = atoi(argv[2]);
    first = 3;
  }
  if (first >= argc) {
    fprintf(stderr, "usage: cwordfreq [-n NTOP] file ...\n");
    return 1;
  }
  void *mr = MR_create(MR_comm_world());
  int me = MR_my_proc(mr);
  uint64_t nwords = MR_map_file(mr, argc - first, &argv[first], 0, 1, 0, read_words, NULL);
  MR_collate(mr, NULL);
  uint64_t nunique = MR_reduce(mr, count, NULL);

  MR_sort_values_flag(mr, -1);
  struct Top t = {ntop, 0};
  void *top = MR_create(MR_comm_world());
  MR_map_mr(top, mr, keep_top, &t);
  MR_gather(top, 1);
  MR_sort_values_flag(top, -1);
  int left = ntop;
  /* scan returns the global pair count (a collective): every rank calls it;
     after gather(1) only rank 0 holds pairs */
  MR_scan_kv(top, print_top, &left);
  if (me == 0) printf("%llu total words, %llu unique words\n", (unsigned long long)nwords, (unsigned long long)nunique);
  MR_destroy(top);
  MR_destroy(mr);
  return 0;
}
