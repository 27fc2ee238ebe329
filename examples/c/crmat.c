/* R-MAT sparse matrix generation through the MR_* C API.
 *
 * The job of the reference's examples/crmat.c: generate N = 2^nlevels rows
 * with about nnonzero entries per row by recursive quadrant choice (a,b,c,d
 * with `fraction` noise), drop duplicates with collate + a "keep first"
 * reduce, loop until enough unique entries exist, then histogram the number
 * of nonzeros per row.
 *
 *   ./crmat nlevels nnonzero a b c d fraction seed
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmapreduce.h"

struct Rmat {
  int nlevels, nprocs;
  uint64_t order, ngenerate;
  double a, b, c, d, fraction;
  uint64_t state; /* per-rank xorshift state */
};

static double urand(struct Rmat *r) {
  r->state ^= r->state << 13;
  r->state ^= r->state >> 7;
  r->state ^= r->state << 17;
  return (double)(r->state >> 11) * (1.0 / 9007199254740992.0);
}

static void generate(int itask, void *kv, void *app) {
  struct Rmat *r = (struct Rmat *)app;
  uint64_t n = r->ngenerate / r->nprocs + ((uint64_t)itask < r->ngenerate % r->nprocs ? 1 : 0);
  for (uint64_t m = 0; m < n; ++m) {
    double a = r->a, b = r->b, c = r->c, d = r->d;
    uint64_t i = 0, j = 0, delta = r->order >> 1;
    for (int level = 0; level < r->nlevels; ++level) {
      double x = urand(r);
      if (x < a) {
      } else if (x < a + b) {
        j += delta;
      } else if (x < a + b + c) {
        i += delta;
      } else {
        i += delta;
        j += delta;
      }
      delta >>= 1;
      if (r->fraction > 0.0) { /* perturb and renormalise */
        a *= 1.0 - r->fraction + 2.0 * r->fraction * urand(r);
        b *= 1.0 - r->fraction + 2.0 * r->fraction * urand(r);
        c *= 1.0 - r->fraction + 2.0 * r->fraction * urand(r);
        d *= 1.0 - r->fraction + 2.0 * r->fraction * urand(r);
        double s = a + b + c + d;
        a /= s;
        b /= s;
        c /= s;
        d /= s;
      }
    }
    uint64_t e[2] = {i, j};
    MR_kv_add(kv, (char *)e, 16, NULL, 0);
  }
}

static void cull(char *key, int kb, char *mv, int nv, int *vb, void *kv, void *app) {
  MR_kv_add(kv, key, kb, NULL, 0);
  (void)mv; (void)nv; (void)vb; (void)app;
}

static void row_of(uint64_t i, char *key, int kb, char *v, int vb, void *kv, void *app) {
  MR_kv_add(kv, key, 8, NULL, 0);
  (void)i; (void)kb; (void)v; (void)vb; (void)app;
}

static void nnz(char *key, int kb, char *mv, int nv, int *vb, void *kv, void *app) {
  int n = nv;
  if (!mv) { int nb; n = (int)MR_multivalue_blocks((void *)vb, &nb); }
  MR_kv_add(kv, (char *)&n, 4, NULL, 0);
  (void)key; (void)kb; (void)app;
}

static void print_histo(char *key, int kb, char *mv, int nv, int *vb, void *app) {
  int n = nv;
  if (!mv) { int nb; n = (int)MR_multivalue_blocks((void *)vb, &nb); }
  printf("%d rows with %d nonzeroes\n", n, *(int *)key);
  (void)kb; (void)app;
}

int main(int argc, char **argv) {
  if (argc != 9) {
    fprintf(stderr, "usage: crmat nlevels nnonzero a b c d fraction seed\n");
    return 1;
  }
  struct Rmat r;
  r.nlevels = atoi(argv[1]);
  uint64_t nnonzero = (uint64_t)atoll(argv[2]);
  r.a = atof(argv[3]); r.b = atof(argv[4]); r.c = atof(argv[5]); r.d = atof(argv[6]);
  r.fraction = atof(argv[7]);
  uint64_t seed = (uint64_t)atoll(argv[8]);
  r.order = 1ull << r.nlevels;
  void *mr = MR_create(MR_comm_world());
  int me = MR_my_proc(mr);
  r.nprocs = MR_num_procs(mr);
  r.state = seed * 0x9E3779B97F4A7C15ull + (uint64_t)me + 1;
  const uint64_t ntotal = r.order * nnonzero;
  uint64_t nremain = ntotal, niter = 0;
  while (nremain) {
    ++niter;
    r.ngenerate = nremain;
    MR_map_add(mr, r.nprocs, generate, &r, 1);
    uint64_t nunique = MR_collate(mr, NULL);
    MR_reduce(mr, cull, NULL);
    nremain = ntotal - nunique;
  }
  if (me == 0)
    printf("%llu rows in matrix\n%llu nonzeroes in matrix\n%llu iterations\n", (unsigned long long)r.order,
           (unsigned long long)ntotal, (unsigned long long)niter);
  /* nonzeros per row, then a histogram of those counts */
  void *rows = MR_create(MR_comm_world());
  MR_map_mr(rows, mr, row_of, NULL);
  MR_collate(rows, NULL);
  MR_reduce(rows, nnz, NULL);
  MR_gather(rows, 1);
  MR_sort_keys_flag(rows, 1);
  MR_convert(rows); /* groups equal counts; fixed-width keys come out in key order */
  MR_scan_kmv(rows, print_histo, NULL); /* collective; only rank 0 has pairs */
  MR_destroy(rows);
  MR_destroy(mr);
  return 0;
}
