// rmat — R-MAT sparse matrix generation + nonzeros-per-row histogram
// (reference examples/rmat.cpp:62-175 and rmat2.cpp: uint64 ids, optional
// MatrixMarket output) on the C++ MapReduce API.
//
//   rmat N Nz a b c d frac seed [OUTFILE] [-v verbosity] [-t timer]
//
// 2^N rows, Nz nonzeros per row on average. Each pass generates the missing
// edges with the Philox R-MAT kernel (counter-based: the edge set depends on
// (seed, edge index) only, not on the number of ranks), then
// collate -> reduce(first) drops duplicates, until all 2^N * Nz are unique
// (the reference's dedup loop, :107-127). Then nonzeros per row:
// map(row) -> collate -> reduce(count) -> map(invert) -> collate ->
// reduce(count) -> gather(1) -> sort_keys(int) -> print.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "apps/app_util.h"
#include "engine/mapreduce.h"

using namespace mrh;

int main(int argc, char** argv) {
  std::vector<std::string> pos;
  int verbosity = 0, timer = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-v") && i + 1 < argc) verbosity = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-t") && i + 1 < argc) timer = std::atoi(argv[++i]);
    else pos.push_back(argv[i]);
  }
  if (pos.size() < 8) {
    std::fprintf(stderr, "Syntax: rmat N Nz a b c d frac seed [outfile] [-v verbosity] [-t timer]\n");
    return 1;
  }
  const int nlevels = std::atoi(pos[0].c_str());
  const uint64_t nnonzero = std::strtoull(pos[1].c_str(), nullptr, 10);
  double a = std::atof(pos[2].c_str()), b = std::atof(pos[3].c_str()), c = std::atof(pos[4].c_str()),
         d = std::atof(pos[5].c_str());
  const double frac = std::atof(pos[6].c_str());
  const uint64_t seed = std::strtoull(pos[7].c_str(), nullptr, 10);
  const std::string outfile = pos.size() > 8 ? pos[8] : "";
  if (nlevels < 1 || nlevels > 40 || a + b + c + d < 0.999 || a + b + c + d > 1.001) {
    std::fprintf(stderr, "ERROR: bad rmat parameters (N in 1..40, a+b+c+d == 1)\n");
    return 1;
  }
  auto comm = Comm::from_env();
  const int me = comm->rank(), np = comm->size();
  const at::Device dev = comm->device();
  const uint64_t order = 1ull << nlevels, ntotal = order * nnonzero;
  {
    MapReduce mr(comm);
    mr.set.verbosity = verbosity;
    mr.set.timer = timer;
    comm->barrier();
    const double t0 = Comm::wtime();
    uint64_t nunique = 0, niter = 0, next_edge = 0;
    while (nunique < ntotal) {
      ++niter;
      const uint64_t want = ntotal - nunique;
      // rank r generates edges [next + want*r/np, next + want*(r+1)/np)
      const uint64_t lo = next_edge + want * me / np, hi = next_edge + want * (me + 1) / np;
      mr.map(np, [&](int, KeyValue& kv) {
        kv.add_kv(map_rmat((int64_t)(hi - lo), nlevels, a, b, c, d, frac, seed, lo, dev));
      }, /*addflag=*/1);
      next_edge += want;
      mr.collate();
      nunique = mr.reduce_builtin("first", "bytes");
    }
    comm->barrier();
    const double t1 = Comm::wtime();
    if (me == 0)
      std::printf("%llu rows in matrix\n%llu nonzeroes in matrix\n%llu iterations, %g secs\n",
                  (unsigned long long)order, (unsigned long long)ntotal, (unsigned long long)niter, t1 - t0);

    if (!outfile.empty()) {
      // MatrixMarket (reference rmat2.cpp): one file per rank, rank 0 writes the header
      const std::string path = np > 1 ? outfile + "." + std::to_string(me) : outfile;
      FILE* f = std::fopen(path.c_str(), "w");
      if (!f) {
        std::fprintf(stderr, "ERROR: cannot write %s\n", path.c_str());
        apps::finish(comm, 1);
      }
      if (me == 0)
        std::fprintf(f, "%%%%MatrixMarket matrix coordinate real general\n%llu %llu %llu\n",
                     (unsigned long long)order, (unsigned long long)order, (unsigned long long)ntotal);
      mr.scan_kv([&](char* k, int, char*, int) {
        const uint64_t* e = (const uint64_t*)k;
        std::fprintf(f, "%llu %llu 1\n", (unsigned long long)e[0] + 1, (unsigned long long)e[1] + 1);
      });
      std::fclose(f);
    }

    // nonzeros per row, then the histogram of those counts
    MapReduce rows(comm);
    rows.map_mr(mr, [](uint64_t, char* k, int, char*, int, KeyValue& kv) { kv.add(k, 8, nullptr, 0); });
    rows.collate();
    rows.reduce([](char*, int, char*, int nv, int* vb, KeyValue& kv) {
      int n = nv;
      if (nv == 0) {
        int nb = 0;
        n = (int)reinterpret_cast<MapReduce*>(vb)->multivalue_blocks(nb);
      }
      kv.add((const char*)&n, 4, nullptr, 0);
    });
    rows.collate();
    rows.reduce_builtin("count", "int32");
    rows.gather(1);
    rows.sort_keys(1);
    rows.scan_kv([](char* k, int, char* v, int) {
      std::printf("%d rows with %d nonzeroes\n", *(int*)v, *(int*)k);
    });
  }
  apps::finish(comm, 0);
}
