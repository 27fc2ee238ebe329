// invertedindex — the reference's GPU application as a native program on the
// C++ MapReduce API (reference cuda/InvertedIndex.cu:140-230, cpu twin
// cpu/InvertedIndex.cpp:49-125): URL -> list of part files linking to it.
//
//   invertedindex INPUT_DIR NUM_FILE [OUTPUT_DIR|NULL] [-v verbosity] [-t timer]
//
// Files INPUT_DIR/part-%05d, 0 <= i < NUM_FILE, are split into contiguous
// blocks, one per rank (the reference's file_each_proc ranges, :278-284).
// One process per GPU (torchrun-style env); the engine device is the GPU
// LOCAL_RANK, or the CPU when no GPU is visible (the cpu/ twin).
//
// Per rank (MI355X design):
//   map     fread each file into a pinned host buffer, hipMemcpyAsync it into
//           one of two HBM staging buffers on a copy stream (double buffered,
//           event-ordered against the map stream), and run the fused URL scan
//           + KV emit kernels (KV(url+NUL, int32 file id)) — no per-URL host
//           loop, no D2H (reference :254-410 copies everything back);
//   aggregate / convert / reduce: RCCL shuffle, hash radix group-by, and the
//           "url\tfile file ...\n" text formatted by one GPU kernel and written
//           with ONE write per rank (the reference opens/appends/closes the
//           output file once per key, :463-513).
// Prints the reference's stage breakdown (Map / Network I/O / Sort/Hash /
// Reduce, chapter_final.pdf Fig. 4/5) and the KV/s and input GB/s.
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "apps/app_util.h"
#include "engine/mapreduce.h"

using namespace mrh;
using apps::file_size;
using apps::hip_check;

namespace {

constexpr int64_t PAD = 64;  // scan windows read past the end of a file

std::string part_name(int i) {
  char b[32];
  std::snprintf(b, sizeof(b), "part-%05d", i);
  return b;
}

struct App {
  std::string dir;
  int nfile = 0, first = 0, last = 0;  // this rank's files [first, last)
  int nprocs = 1;
  int64_t in_bytes = 0;
};

// one map task per rank: stream this rank's files through HBM
void map_files(App& app, KeyValue& kv, at::Device dev) {
  const int nf = app.last - app.first;
  if (nf <= 0) return;
  // one rank: group each part file as it arrives (the aggregate that follows
  // is the identity, so convert finds the group-by done; keyvalue.h)
  if (app.nprocs == 1) kv.enable_grouping();
  std::vector<int64_t> sizes(nf);
  int64_t maxlen = 0;
  for (int i = 0; i < nf; ++i) {
    sizes[i] = file_size(app.dir + "/" + part_name(app.first + i));
    if (sizes[i] < 0) {
      std::fprintf(stderr, "ERROR: cannot open %s/%s\n", app.dir.c_str(), part_name(app.first + i).c_str());
      std::exit(1);
    }
    maxlen = std::max(maxlen, sizes[i]);
  }
  auto u8 = at::TensorOptions().dtype(at::kByte);
  auto read_into = [&](int i, uint8_t* dst) {
    FILE* f = std::fopen((app.dir + "/" + part_name(app.first + i)).c_str(), "rb");
    const size_t got = std::fread(dst, 1, (size_t)sizes[i], f);
    std::fclose(f);
    app.in_bytes += (int64_t)got;
    MapReduce::rsize += (int64_t)got;
    std::memset(dst + got, 0, PAD);
  };
  if (!dev.is_cuda()) {
    at::Tensor buf = at::empty({maxlen + PAD}, u8);
    for (int i = 0; i < nf; ++i) {
      read_into(i, buf.data_ptr<uint8_t>());
      kv.add_kv(map_urls(buf, sizes[i], app.first + i));
    }
    return;
  }
  // two pinned host buffers + two HBM buffers; file i+1 is read and copied
  // while the kernels of file i run
  at::Tensor host[2], devb[2];
  hipEvent_t ready[2], freed[2];
  for (int b = 0; b < 2; ++b) {
    host[b] = at::empty({maxlen + PAD}, u8.pinned_memory(true));
    devb[b] = at::empty({maxlen + PAD}, u8.device(dev));
    hip_check(hipEventCreateWithFlags(&ready[b], hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&freed[b], hipEventDisableTiming), "hipEventCreate");
  }
  hipStream_t main_s = at::hip::getCurrentHIPStream();
  hipStream_t copy_s = at::hip::getStreamFromPool().stream();
  auto issue = [&](int i) {
    const int b = i & 1;
    if (i >= 2) {
      hip_check(hipEventSynchronize(freed[b]), "hipEventSynchronize");  // host buffer reusable
      hip_check(hipStreamWaitEvent(copy_s, freed[b], 0), "hipStreamWaitEvent");
    }
    read_into(i, host[b].data_ptr<uint8_t>());
    hip_check(hipMemcpyAsync(devb[b].data_ptr(), host[b].data_ptr(), sizes[i] + PAD, hipMemcpyHostToDevice, copy_s),
              "hipMemcpyAsync");
    hip_check(hipEventRecord(ready[b], copy_s), "hipEventRecord");
  };
  issue(0);
  for (int i = 0; i < nf; ++i) {
    const int b = i & 1;
    hip_check(hipStreamWaitEvent(main_s, ready[b], 0), "hipStreamWaitEvent");
    kv.add_kv(map_urls(devb[b], sizes[i], app.first + i));
    hip_check(hipEventRecord(freed[b], main_s), "hipEventRecord");
    if (i + 1 < nf) issue(i + 1);
  }
  hip_check(hipStreamSynchronize(main_s), "hipStreamSynchronize");
  for (int b = 0; b < 2; ++b) {
    hipEventDestroy(ready[b]);
    hipEventDestroy(freed[b]);
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<std::string> pos;
  int verbosity = 0, timer = 0;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "-v") && i + 1 < argc) verbosity = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-t") && i + 1 < argc) timer = std::atoi(argv[++i]);
    else pos.push_back(argv[i]);
  }
  if (pos.size() < 2) {
    std::fprintf(stderr, "Syntax: invertedindex INPUT_DIR NUM_FILE [OUTPUT_DIR|NULL] [-v verbosity] [-t timer]\n");
    return 1;
  }
  auto comm = Comm::from_env();
  const int me = comm->rank(), np = comm->size();
  App app;
  app.dir = pos[0];
  app.nfile = std::atoi(pos[1].c_str());
  app.first = (int)((int64_t)app.nfile * me / np);
  app.last = (int)((int64_t)app.nfile * (me + 1) / np);
  app.nprocs = np;
  const std::string outdir = pos.size() > 2 ? pos[2] : "NULL";
  const at::Device dev = comm->device();

  // file names by global id, for the reduce epilogue
  std::string names;
  std::vector<int64_t> noff{0};
  for (int i = 0; i < app.nfile; ++i) {
    names += part_name(i);
    noff.push_back((int64_t)names.size());
  }
  at::Tensor names_t = at::empty({(int64_t)names.size()}, at::kByte);
  std::memcpy(names_t.data_ptr(), names.data(), names.size());
  at::Tensor noff_t = at::tensor(noff, at::kLong);
  names_t = names_t.to(dev);
  noff_t = noff_t.to(dev);

  auto sync = [&]() {
    if (dev.is_cuda()) hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    comm->barrier();
  };
  {
    MapReduce mr(comm);
    mr.set.verbosity = verbosity;
    mr.set.timer = timer;
    sync();
    double t[5];
    t[0] = Comm::wtime();
    const uint64_t nurl = mr.map(np, [&](int, KeyValue& kv) { map_files(app, kv, dev); });
    sync();
    t[1] = Comm::wtime();
    mr.aggregate();
    sync();
    t[2] = Comm::wtime();
    const uint64_t nunique = mr.convert();
    sync();
    t[3] = Comm::wtime();
    at::Tensor text;
    mr.reduce_batch([&](const KMV& kmv, KeyValue&) { text = inverted_index_format(kmv, names_t, noff_t); });
    at::Tensor host = text.defined() ? text.to(at::kCPU) : at::empty({0}, at::kByte);
    if (outdir != "NULL") {
      const std::string path = outdir + "/InvertedIndex-" + std::to_string(np) + "-" + std::to_string(me);
      FILE* f = std::fopen(path.c_str(), "wb");
      if (!f) {
        std::fprintf(stderr, "ERROR: cannot write %s\n", path.c_str());
        apps::finish(comm, 1);
      }
      std::fwrite(host.data_ptr(), 1, (size_t)host.numel(), f);
      std::fclose(f);
      MapReduce::wsize += host.numel();
    }
    sync();
    t[4] = Comm::wtime();
    const double in_bytes = (double)comm->allreduce(app.in_bytes, Comm::SUM);
    if (me == 0) {
      const double tot = t[4] - t[0];
      std::printf("InvertedIndex: %d files, %.3f MB, %llu URL KVs, %llu unique URLs on %d procs (%s)\n", app.nfile,
                  in_bytes / 1e6, (unsigned long long)nurl, (unsigned long long)nunique, np,
                  dev.is_cuda() ? "gpu" : "cpu");
      std::printf("Map %.6f s, Network I/O %.6f s, Sort/Hash %.6f s, Reduce %.6f s, total %.6f s\n", t[1] - t[0],
                  t[2] - t[1], t[3] - t[2], t[4] - t[3], tot);
      std::printf("Throughput: %.3f M KV/s, %.3f GB/s input\n", nurl / tot / 1e6, in_bytes / tot / 1e9);
    }
  }
  apps::finish(comm, 0);
}
