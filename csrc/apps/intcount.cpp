// intcount — integer counting (reference cpu/IntCount.cpp:150-190, the GPMR
// IntegerCount workload of chapter_final.pdf Fig. 6b) as a native program.
//
//   intcount FILE [NBYTES] [-noreduce] [-v verbosity] [-t timer]
//
// Every rank reads NBYTES (default: the whole file; the reference reads
// 128 MB = 32M ints) of raw 4-byte ints from FILE (or FILE.<rank> when that
// exists), emits KV(int, 1) for each, then aggregate -> convert -> reduce
// (count). The reference's host loop of 32M kv->add calls (:179-180) is one
// H2D copy + a fixed-width device KV here; convert is an exact-key radix
// sort and the count is a segmented reduce kernel.
#include <ATen/hip/HIPContext.h>

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
  bool do_reduce = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-v") && i + 1 < argc) verbosity = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-t") && i + 1 < argc) timer = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-noreduce")) do_reduce = false;
    else pos.push_back(argv[i]);
  }
  if (pos.empty()) {
    std::fprintf(stderr, "Syntax: intcount FILE [NBYTES] [-noreduce] [-v verbosity] [-t timer]\n");
    return 1;
  }
  auto comm = Comm::from_env();
  const int me = comm->rank(), np = comm->size();
  const at::Device dev = comm->device();
  std::string path = pos[0] + "." + std::to_string(me);
  if (apps::file_size(path) < 0) path = pos[0];
  int64_t nbytes = apps::file_size(path);
  if (nbytes < 0) {
    std::fprintf(stderr, "ERROR: Could not query file size of %s\n", path.c_str());
    apps::finish(comm, 1);
  }
  if (pos.size() > 1) nbytes = std::min<int64_t>(nbytes, std::atoll(pos[1].c_str()));
  nbytes &= ~int64_t(3);
  at::Tensor host = at::empty({nbytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(dev.is_cuda()));
  {
    FILE* f = std::fopen(path.c_str(), "rb");
    const size_t got = std::fread(host.data_ptr(), 1, (size_t)nbytes, f);
    std::fclose(f);
    if ((int64_t)got != nbytes) {
      std::fprintf(stderr, "ERROR: short read of %s\n", path.c_str());
      apps::finish(comm, 1);
    }
    MapReduce::rsize += nbytes;
  }
  auto sync = [&]() {
    if (dev.is_cuda()) apps::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    comm->barrier();
  };
  {
    MapReduce mr(comm);
    mr.set.verbosity = verbosity;
    mr.set.timer = timer;
    sync();
    double t[5];
    t[0] = Comm::wtime();
    const uint64_t nkv = mr.map(np, [&](int, KeyValue& kv) {
      at::Tensor keys = host.to(dev, /*non_blocking=*/true);
      const int64_t n = nbytes / 4;
      at::Tensor ones = at::ones({n}, at::TensorOptions().dtype(at::kInt).device(dev));
      kv.add_kv(make_kv(keys, c10::nullopt, ones, c10::nullopt, n, dev));
    });
    sync();
    t[1] = Comm::wtime();
    mr.aggregate();
    sync();
    t[2] = Comm::wtime();
    const uint64_t nunique = mr.convert();
    sync();
    t[3] = Comm::wtime();
    if (do_reduce) mr.reduce_builtin("count", "int32");
    sync();
    t[4] = Comm::wtime();
    if (me == 0) {
      const double tot = t[4] - t[0];
      std::printf("IntCount: %llu ints, %llu unique on %d procs (%s)\n", (unsigned long long)nkv,
                  (unsigned long long)nunique, np, dev.is_cuda() ? "gpu" : "cpu");
      std::printf("Map %.6f s, Network I/O %.6f s, Sort/Hash %.6f s, Reduce %.6f s, total %.6f s\n", t[1] - t[0],
                  t[2] - t[1], t[3] - t[2], t[4] - t[3], tot);
      std::printf("Throughput: %.3f M KV/s\n", nkv / tot / 1e6);
    }
    // checksum: the counts add up to the number of ints
    if (do_reduce) {
      int64_t local = 0;
      mr.flatten();
      if (mr.kv && mr.kv->n) local = mr.kv->vdata.view(at::kInt).sum().item<int64_t>();
      const int64_t tot = comm->allreduce(local, Comm::SUM);
      if (me == 0) std::printf("Counts sum: %lld\n", (long long)tot);
    }
  }
  apps::finish(comm, 0);
}
