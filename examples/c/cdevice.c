/* Device functors through the MR_* C API: the map and the reduce are HIP
 * device code (strings), compiled at run time for the GPU by the engine
 * (csrc/engine/devfn.h) — no host callback touches a pair.
 *
 * ntask tasks each emit (t % nkey, 1); collate; a device reduce sums each
 * key's values into an int64; a device sort-key functor orders the keys by
 * count. Prints the number of keys and the sum of the sums (= ntask), then the
 * count of key 0 (= ceil(ntask / nkey)).
 *
 *   ./cdevice ntask nkey      (on a GPU MapReduce)
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmapreduce.h"

static const char *MAP_SRC =
    "__device__ void mr_map(mrd::Bytes key, mrd::Bytes value, long long t, mrd::Emit& out) {\n"
    "  out.emit((long long)(t % NKEY), (int)1);\n"
    "}\n";

static const char *REDUCE_SRC =
    "__device__ void mr_reduce(mrd::Bytes key, mrd::Values vals, mrd::Emit& out) {\n"
    "  long long s = 0;\n"
    "  for (long long i = 0; i < vals.n; ++i) s += vals.get<int>(i);\n"
    "  out.emit(key.as<long long>(), s);\n"
    "}\n";

struct Totals {
  int64_t nkey, sum, count0, first;
};

static void tally(char *key, int kb, char *value, int vb, void *app) {
  struct Totals *t = (struct Totals *)app;
  int64_t k, v;
  memcpy(&k, key, 8);
  memcpy(&v, value, 8);
  if (t->nkey == 0) t->first = v;
  t->nkey++;
  t->sum += v;
  if (k == 0) t->count0 = v;
}

int main(int argc, char **argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: cdevice ntask nkey\n");
    return 1;
  }
  const uint64_t ntask = strtoull(argv[1], NULL, 10);
  const long nkey = atol(argv[2]);
  char map_src[512];
  snprintf(map_src, sizeof(map_src), "#define NKEY %ldLL\n%s", nkey, MAP_SRC);
  void *mr = MR_create(MR_comm_world());
  MR_map_device_tasks(mr, ntask, map_src, 0);
  MR_collate(mr, NULL);
  MR_reduce_device(mr, REDUCE_SRC);
  /* order the keys by their count, largest first (a sort on the values) */
  MR_sort_values_device(mr, "__device__ unsigned long long mr_sortkey(mrd::Bytes v) {\n"
                            "  return ~(unsigned long long)v.as<long long>();\n}\n", 64);
  struct Totals t = {0, 0, 0, 0};
  MR_scan_kv(mr, tally, &t);
  if (MR_my_proc(mr) == 0)
    printf("keys %lld sum %lld count0 %lld first %lld\n", (long long)t.nkey, (long long)t.sum, (long long)t.count0,
           (long long)t.first);
  MR_destroy(mr);
  return 0;
}
