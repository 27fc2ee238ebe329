// C ABI over mrh::MapReduce (reference src/cmapreduce.cpp:23-462). The MR
// handle IS the MapReduce*, so the multi-block protocol works unchanged: a
// reduce callback that receives multivalue == NULL casts valuebytes back to
// the MR handle and calls MR_multivalue_blocks/MR_multivalue_block.
#include "cmapreduce.h"

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../engine/mapreduce.h"

using mrh::KeyValue;
using mrh::MapReduce;

namespace {

std::string g_err;
int g_mode = 0;
std::mutex g_world_mu;
std::shared_ptr<mrh::Comm> g_world;

// A C program exits through exit() -> atexit handlers -> DSO destructors. On
// ROCm 7 the HIP fat-binary unregistration of libtorch_hip can then crash
// inside the HIP runtime (hipUnregisterFatBinary after the runtime's own
// teardown). Once the engine runs on a GPU, the C API therefore finishes the
// process itself: flush stdio and _exit with the program's status, from an
// on_exit handler that runs before the library destructors. Handlers the
// program registers after its first MR_* call still run first.
void finish_process(int status, void*) {
  std::fflush(nullptr);
  std::_Exit(status);
}

std::shared_ptr<mrh::Comm> world() {
  std::lock_guard<std::mutex> l(g_world_mu);
  if (!g_world) {
    g_world = mrh::Comm::from_env();
    if (g_world->device().is_cuda()) on_exit(finish_process, nullptr);
    // registered last so it runs first: rank 0 (the rendezvous server) waits
    // for every rank to be done with the store before the process ends
    // (a non-zero exit status is a failure: peers are told, not released)
    if (g_world->size() > 1)
      on_exit([](int st, void*) {
        if (st != 0) g_world->poison("process exited with status " + std::to_string(st));
        else g_world->shutdown();
      }, nullptr);
  }
  return g_world;
}

template <typename F, typename R>
R guard(F&& f, R bad) {
  try {
    return f();
  } catch (const std::exception& e) {
    g_err = e.what();
    if (g_mode) return bad;
    // reference Error::one -> MPI_Abort (src/error.cpp:47-57): the whole job
    // ends; peers are told through the communicator and fail within seconds
    std::fprintf(stderr, "ERROR: %s\n", e.what());
    std::fflush(nullptr);
    if (g_world) g_world->poison(e.what());
    std::_Exit(1);
  }
}
template <typename F>
void guardv(F&& f) {
  guard([&]() { f(); return 0; }, 0);
}

MapReduce* M(void* p) { return static_cast<MapReduce*>(p); }
std::vector<std::string> strs(int n, char** s) { return std::vector<std::string>(s, s + n); }

}  // namespace

namespace mrh {
// the job communicator shared by the C APIs (MR_*, oink_*) and the oink executable
std::shared_ptr<Comm> capi_world() { return world(); }
}  // namespace mrh

extern "C" {

void* MR_comm_world(void) {
  return guard([]() -> void* { return world().get(); }, (void*)nullptr);
}

void* MR_create(void* comm) {
  return guard(
      [&]() -> void* {
        auto w = world();
        if (comm && comm != w.get()) throw std::runtime_error("MR_create: unknown communicator handle");
        return new MapReduce(w);
      },
      (void*)nullptr);
}
void* MR_create_mpi(void) { return MR_create(nullptr); }
void* MR_create_mpi_finalize(void) { return MR_create(nullptr); }
void MR_destroy(void* p) { delete M(p); }
int MR_my_proc(void* p) { return M(p)->my_proc(); }
int MR_num_procs(void* p) { return M(p)->num_procs(); }

void* MR_copy(void* p) {
  return guard([&]() -> void* { return M(p)->copy().release(); }, (void*)nullptr);
}

uint64_t MR_add(void* p, void* p2) { return guard([&] { return M(p)->add(*M(p2)); }, (uint64_t)0); }

static mrh::HashFn hashfn(int (*h)(char*, int)) {
  if (!h) return nullptr;
  return [h](char* k, int kb) { return h(k, kb); };
}
uint64_t MR_aggregate(void* p, int (*h)(char*, int)) {
  return guard([&] { return M(p)->aggregate(hashfn(h)); }, (uint64_t)0);
}
uint64_t MR_broadcast(void* p, int root) { return guard([&] { return M(p)->broadcast(root); }, (uint64_t)0); }
uint64_t MR_clone(void* p) { return guard([&] { return M(p)->clone(); }, (uint64_t)0); }
uint64_t MR_close(void* p) { return guard([&] { return M(p)->close(); }, (uint64_t)0); }
uint64_t MR_collapse(void* p, char* key, int kb) {
  return guard([&] { return M(p)->collapse(key, kb); }, (uint64_t)0);
}
uint64_t MR_collate(void* p, int (*h)(char*, int)) {
  return guard([&] { return M(p)->collate(hashfn(h)); }, (uint64_t)0);
}

using CReduce = void (*)(char*, int, char*, int, int*, void*, void*);
static mrh::ReduceFn reducefn(CReduce f, void* app) {
  return [f, app](char* k, int kb, char* mv, int nv, int* vb, KeyValue& kv) { f(k, kb, mv, nv, vb, &kv, app); };
}
uint64_t MR_compress(void* p, CReduce f, void* app) {
  return guard([&] { return M(p)->compress(reducefn(f, app)); }, (uint64_t)0);
}
uint64_t MR_convert(void* p) { return guard([&] { return M(p)->convert(); }, (uint64_t)0); }
uint64_t MR_gather(void* p, int n) { return guard([&] { return M(p)->gather(n); }, (uint64_t)0); }

uint64_t MR_map(void* p, int nmap, void (*f)(int, void*, void*), void* app) { return MR_map_add(p, nmap, f, app, 0); }
uint64_t MR_map_add(void* p, int nmap, void (*f)(int, void*, void*), void* app, int addflag) {
  return guard([&] { return M(p)->map(nmap, [f, app](int t, KeyValue& kv) { f(t, &kv, app); }, addflag); },
               (uint64_t)0);
}
uint64_t MR_map_file(void* p, int nstr, char** s, int self, int recurse, int readfile,
                     void (*f)(int, char*, void*, void*), void* app) {
  return MR_map_file_add(p, nstr, s, self, recurse, readfile, f, app, 0);
}
uint64_t MR_map_file_add(void* p, int nstr, char** s, int self, int recurse, int readfile,
                         void (*f)(int, char*, void*, void*), void* app, int addflag) {
  return guard(
      [&] {
        return M(p)->map_file(
            strs(nstr, s), self, recurse, readfile,
            [f, app](int t, const char* fn, KeyValue& kv) { f(t, const_cast<char*>(fn), &kv, app); }, addflag);
      },
      (uint64_t)0);
}
using CChunk = void (*)(int, char*, int, void*, void*);
uint64_t MR_map_file_char(void* p, int nmap, int nstr, char** s, int recurse, int readflag, char sep, int delta,
                          CChunk f, void* app) {
  return MR_map_file_char_add(p, nmap, nstr, s, recurse, readflag, sep, delta, f, app, 0);
}
uint64_t MR_map_file_char_add(void* p, int nmap, int nstr, char** s, int recurse, int readflag, char sep, int delta,
                              CChunk f, void* app, int addflag) {
  return guard(
      [&] {
        return M(p)->map_file_char(
            nmap, strs(nstr, s), 0, recurse, readflag, sep, delta,
            [f, app](int t, char* str, int n, KeyValue& kv) { f(t, str, n, &kv, app); }, addflag);
      },
      (uint64_t)0);
}
uint64_t MR_map_file_str(void* p, int nmap, int nstr, char** s, int recurse, int readflag, char* sep, int delta,
                         CChunk f, void* app) {
  return MR_map_file_str_add(p, nmap, nstr, s, recurse, readflag, sep, delta, f, app, 0);
}
uint64_t MR_map_file_str_add(void* p, int nmap, int nstr, char** s, int recurse, int readflag, char* sep, int delta,
                             CChunk f, void* app, int addflag) {
  return guard(
      [&] {
        return M(p)->map_file_str(
            nmap, strs(nstr, s), 0, recurse, readflag, sep, delta,
            [f, app](int t, char* str, int n, KeyValue& kv) { f(t, str, n, &kv, app); }, addflag);
      },
      (uint64_t)0);
}
using CMapMR = void (*)(uint64_t, char*, int, char*, int, void*, void*);
uint64_t MR_map_mr(void* p, void* p2, CMapMR f, void* app) { return MR_map_mr_add(p, p2, f, app, 0); }
uint64_t MR_map_mr_add(void* p, void* p2, CMapMR f, void* app, int addflag) {
  return guard(
      [&] {
        return M(p)->map_mr(
            *M(p2), [f, app](uint64_t i, char* k, int kb, char* v, int vb, KeyValue& kv) { f(i, k, kb, v, vb, &kv, app); },
            addflag);
      },
      (uint64_t)0);
}

void MR_open(void* p) { MR_open_add(p, 0); }
void MR_open_add(void* p, int addflag) { guardv([&] { M(p)->open(addflag); }); }
void* MR_kv_open(void* p) {
  return guard([&]() -> void* { return &M(p)->kv_open(); }, (void*)nullptr);
}
void MR_print(void* p, int proc, int nstride, int kflag, int vflag) {
  guardv([&] { M(p)->print(proc, nstride, kflag, vflag); });
}
void MR_print_file(void* p, char* file, int fflag, int proc, int nstride, int kflag, int vflag) {
  guardv([&] { M(p)->print(file, fflag, proc, nstride, kflag, vflag); });
}

uint64_t MR_reduce(void* p, CReduce f, void* app) {
  return guard([&] { return M(p)->reduce(reducefn(f, app)); }, (uint64_t)0);
}
uint64_t MR_reduce_builtin(void* p, const char* op, const char* dtype) {
  return guard([&] { return M(p)->reduce_builtin(op, dtype ? dtype : "int32"); }, (uint64_t)0);
}
uint64_t MR_map_device(void* p, void* src, const char* code, int addflag) {
  return guard([&] { return M(p)->map_device(*M(src), code, addflag); }, (uint64_t)0);
}
uint64_t MR_map_device_tasks(void* p, uint64_t ntask, const char* code, int addflag) {
  return guard([&] { return M(p)->map_device_tasks((int64_t)ntask, code, addflag); }, (uint64_t)0);
}
uint64_t MR_reduce_device(void* p, const char* code) {
  return guard([&] { return M(p)->reduce_device(code); }, (uint64_t)0);
}
uint64_t MR_compress_device(void* p, const char* code) {
  return guard([&] { return M(p)->compress_device(code); }, (uint64_t)0);
}
uint64_t MR_sort_keys_device(void* p, const char* code, int bits) {
  return guard([&] { return M(p)->sort_keys_device(code, bits); }, (uint64_t)0);
}
uint64_t MR_sort_values_device(void* p, const char* code, int bits) {
  return guard([&] { return M(p)->sort_values_device(code, bits); }, (uint64_t)0);
}
uint64_t MR_multivalue_blocks(void* p, int* nblock) {
  int nb = 0;
  uint64_t n = M(p)->multivalue_blocks(nb);
  if (nblock) *nblock = nb;
  return n;
}
void MR_multivalue_block_select(void* p, int which) { M(p)->multivalue_block_select(which); }
int MR_multivalue_block(void* p, int iblock, char** mv, int** vb) {
  return guard([&] { return M(p)->multivalue_block(iblock, mv, vb); }, 0);
}
uint64_t MR_scan_kv(void* p, void (*f)(char*, int, char*, int, void*), void* app) {
  return guard([&] { return M(p)->scan_kv([f, app](char* k, int kb, char* v, int vb) { f(k, kb, v, vb, app); }); },
               (uint64_t)0);
}
uint64_t MR_scan_kmv(void* p, void (*f)(char*, int, char*, int, int*, void*), void* app) {
  return guard(
      [&] {
        return M(p)->scan_kmv([f, app](char* k, int kb, char* mv, int nv, int* vb) { f(k, kb, mv, nv, vb, app); });
      },
      (uint64_t)0);
}

uint64_t MR_scrunch(void* p, int n, char* key, int kb) {
  return guard([&] { return M(p)->scrunch(n, key, kb); }, (uint64_t)0);
}
static mrh::CompareFn cmpfn(int (*c)(char*, int, char*, int)) {
  return [c](char* a, int al, char* b, int bl) { return c(a, al, b, bl); };
}
uint64_t MR_sort_keys(void* p, int (*c)(char*, int, char*, int)) {
  return guard([&] { return M(p)->sort_keys(cmpfn(c)); }, (uint64_t)0);
}
uint64_t MR_sort_keys_flag(void* p, int flag) { return guard([&] { return M(p)->sort_keys(flag); }, (uint64_t)0); }
uint64_t MR_sort_values(void* p, int (*c)(char*, int, char*, int)) {
  return guard([&] { return M(p)->sort_values(cmpfn(c)); }, (uint64_t)0);
}
uint64_t MR_sort_values_flag(void* p, int flag) { return guard([&] { return M(p)->sort_values(flag); }, (uint64_t)0); }
uint64_t MR_sort_multivalues(void* p, int (*c)(char*, int, char*, int)) {
  return guard([&] { return M(p)->sort_multivalues(cmpfn(c)); }, (uint64_t)0);
}
uint64_t MR_sort_multivalues_flag(void* p, int flag) {
  return guard([&] { return M(p)->sort_multivalues(flag); }, (uint64_t)0);
}

void MR_save(void* p, const char* path) { guardv([&] { M(p)->save(path); }); }
uint64_t MR_load(void* p, const char* path) { return guard([&] { return M(p)->load(path); }, (uint64_t)0); }

uint64_t MR_kv_stats(void* p, int level) { return guard([&] { return M(p)->kv_stats(level); }, (uint64_t)0); }
uint64_t MR_kmv_stats(void* p, int level) { return guard([&] { return M(p)->kmv_stats(level); }, (uint64_t)0); }
void MR_cummulative_stats(void* p, int level, int reset) { guardv([&] { M(p)->cummulative_stats(level, reset); }); }

void MR_set_mapstyle(void* p, int v) { M(p)->set.mapstyle = v; }
void MR_set_all2all(void* p, int v) { M(p)->set.all2all = v; }
void MR_set_verbosity(void* p, int v) { M(p)->set.verbosity = v; }
void MR_set_timer(void* p, int v) { M(p)->set.timer = v; }
void MR_set_memsize(void* p, int v) { M(p)->set.memsize = v; }
void MR_set_minpage(void* p, int v) { M(p)->set.minpage = v; }
void MR_set_maxpage(void* p, int v) { M(p)->set.maxpage = v; }
void MR_set_freepage(void* p, int v) { M(p)->set.freepage = v; }
void MR_set_outofcore(void* p, int v) { M(p)->set.outofcore = v; }
void MR_set_zeropage(void* p, int v) { M(p)->set.zeropage = v; }
void MR_set_keyalign(void* p, int v) { M(p)->set.keyalign = v; }
void MR_set_valuealign(void* p, int v) { M(p)->set.valuealign = v; }
void MR_set_fpath(void* p, char* s) { M(p)->set_fpath(s ? s : "."); }
void MR_set_chunk_bytes(void* p, int64_t v) { M(p)->set.chunk_bytes = v; }
void MR_set_hbm_budget(void* p, int64_t v) { M(p)->set.hbm_budget = v; }
void MR_set_host_budget(void* p, int64_t v) { M(p)->set.host_budget = v; }
void MR_set_pipeline(void* p, int v) { M(p)->set.pipeline = v; }

void MR_kv_add(void* kv, char* k, int kb, char* v, int vb) { static_cast<KeyValue*>(kv)->add(k, kb, v, vb); }
void MR_kv_add_multi_static(void* kv, int n, char* k, int kb, char* v, int vb) {
  static_cast<KeyValue*>(kv)->add((int64_t)n, k, (int64_t)kb, v, (int64_t)vb);
}
void MR_kv_add_multi_dynamic(void* kv, int n, char* k, int* kb, char* v, int* vb) {
  static_cast<KeyValue*>(kv)->add((int64_t)n, k, kb, v, vb);
}

const char* MR_last_error(void) { return g_err.c_str(); }
void MR_set_error_mode(int m) { g_mode = m; }

}  // extern "C"
