// wordfreq — word frequencies with a top-N list, the canonical MR-MPI example
// (reference examples/wordfreq.cpp:42-130, oink/wordfreq.cpp:40-90) on the
// C++ MapReduce API.
//
//   wordfreq [-n NTOP] [-v verbosity] [-t timer] FILE_OR_DIR ...
//
// map_file hands each rank its files; each file goes to HBM once and the
// in-mapper combining kernels (WordCounter, csrc/kernels/wordcount.hip)
// tokenize and count it on the device, emitting KV(word+NUL, count) once per
// distinct word of the file (the reference strtok()s on the host and adds
// every word, :122-127). collate (hash partition + RCCL all-to-all +
// group-by) -> reduce(sum) -> sort_values(-1) -> per-rank top N ->
// gather(1) -> sort_values(-1) -> print.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "apps/app_util.h"
#include "engine/mapreduce.h"
#include "engine/wordcount.h"

using namespace mrh;

int main(int argc, char** argv) {
  std::vector<std::string> files;
  int ntop = 10, verbosity = 0, timer = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-n") && i + 1 < argc) ntop = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-v") && i + 1 < argc) verbosity = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-t") && i + 1 < argc) timer = std::atoi(argv[++i]);
    else files.push_back(argv[i]);
  }
  if (files.empty()) {
    std::fprintf(stderr, "Syntax: wordfreq [-n NTOP] [-v verbosity] [-t timer] file1 dir1 ...\n");
    return 1;
  }
  auto comm = Comm::from_env();
  const int me = comm->rank();
  const at::Device dev = comm->device();
  {
    MapReduce mr(comm);
    mr.set.verbosity = verbosity;
    mr.set.timer = timer;
    comm->barrier();
    const double t0 = Comm::wtime();
    int64_t local_words = 0;
    mr.map_file(files, 0, 1, 0, [&](int, const char* fname, KeyValue& kv) {
      const int64_t n = apps::file_size(fname);
      if (n < 0) {
        std::fprintf(stderr, "ERROR: cannot open %s\n", fname);
        std::exit(1);
      }
      at::Tensor host = at::zeros({n + 64}, at::TensorOptions().dtype(at::kByte).pinned_memory(dev.is_cuda()));
      FILE* f = std::fopen(fname, "rb");
      const size_t got = std::fread(host.data_ptr(), 1, (size_t)n, f);
      std::fclose(f);
      MapReduce::rsize += (int64_t)got;
      WordCounter wc(dev);
      wc.add(host.to(dev, /*non_blocking=*/true), (int64_t)got);
      local_words += wc.words();
      kv.add_kv(wc.finish());
    });
    const uint64_t nwords = (uint64_t)comm->allreduce(local_words, Comm::SUM);
    mr.collate();
    const uint64_t nunique = mr.reduce_builtin("sum", "int32");
    comm->barrier();
    const double t1 = Comm::wtime();

    mr.sort_values(-1);
    MapReduce top(comm);
    int seen = 0;
    top.map_mr(mr, [&](uint64_t, char* k, int kb, char* v, int vb, KeyValue& kv) {
      if (seen++ < ntop) kv.add(k, kb, v, vb);
    });
    top.gather(1);
    top.sort_values(-1);
    int left = ntop;
    top.scan_kv([&](char* k, int, char* v, int) {
      if (left-- > 0) std::printf("%d %s\n", *(int*)v, k);
    });
    if (me == 0) {
      std::printf("%llu total words, %llu unique words\n", (unsigned long long)nwords, (unsigned long long)nunique);
      std::printf("Time to process %d files on %d procs = %g (secs)\n", mr.mapfilecount, comm->size(), t1 - t0);
    }
  }
  apps::finish(comm, 0);
}
