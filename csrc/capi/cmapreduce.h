/* C interface to the gpu_mapreduce_amd native MapReduce engine.
 *
 * Same MR_* entry points and callback shapes as MR-MPI's C API (reference
 * src/cmapreduce.h:24-148), minus the MPI dependency: an MR is created on the
 * job communicator bootstrapped from torchrun-style environment variables
 * (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR, MASTER_PORT). One process per
 * GPU; WORLD_SIZE > 1 shuffles over RCCL (xGMI). Data lives in HBM; host
 * callbacks see the reference's byte views.
 *
 * Differences, all deliberate:
 *  - MR_create takes an opaque communicator from MR_comm_world() (NULL = the
 *    same); MR_create_mpi / MR_create_mpi_finalize are kept as aliases;
 *  - MR_map_file* take `char **strings` (the reference header says `char *`
 *    while its implementation uses `char **`);
 *  - MR_multivalue_blocks returns the value count and the block count through
 *    `nblock` (the reference header and implementation disagree, :104 vs :278).
 */
#ifndef MRHIP_CMAPREDUCE_H
#define MRHIP_CMAPREDUCE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void *MR_comm_world(void);
void *MR_create(void *comm);
void *MR_create_mpi(void);
void *MR_create_mpi_finalize(void);
void MR_destroy(void *MRptr);
int MR_my_proc(void *MRptr);
int MR_num_procs(void *MRptr);

void *MR_copy(void *MRptr);

uint64_t MR_add(void *MRptr, void *MRptr2);
uint64_t MR_aggregate(void *MRptr, int (*myhash)(char *, int));
uint64_t MR_broadcast(void *MRptr, int root);
uint64_t MR_clone(void *MRptr);
uint64_t MR_close(void *MRptr);
uint64_t MR_collapse(void *MRptr, char *key, int keybytes);
uint64_t MR_collate(void *MRptr, int (*myhash)(char *, int));
uint64_t MR_compress(void *MRptr, void (*mycompress)(char *, int, char *, int, int *, void *KVptr, void *APPptr),
                     void *APPptr);
uint64_t MR_convert(void *MRptr);
uint64_t MR_gather(void *MRptr, int numprocs);

uint64_t MR_map(void *MRptr, int nmap, void (*mymap)(int, void *KVptr, void *APPptr), void *APPptr);
uint64_t MR_map_add(void *MRptr, int nmap, void (*mymap)(int, void *KVptr, void *APPptr), void *APPptr,
                    int addflag);
uint64_t MR_map_file(void *MRptr, int nstr, char **strings, int self, int recurse, int readfile,
                     void (*mymap)(int, char *, void *KVptr, void *APPptr), void *APPptr);
uint64_t MR_map_file_add(void *MRptr, int nstr, char **strings, int self, int recurse, int readfile,
                         void (*mymap)(int, char *, void *KVptr, void *APPptr), void *APPptr, int addflag);
uint64_t MR_map_file_char(void *MRptr, int nmap, int nstr, char **strings, int recurse, int readflag, char sepchar,
                          int delta, void (*mymap)(int, char *, int, void *KVptr, void *APPptr), void *APPptr);
uint64_t MR_map_file_char_add(void *MRptr, int nmap, int nstr, char **strings, int recurse, int readflag,
                              char sepchar, int delta, void (*mymap)(int, char *, int, void *KVptr, void *APPptr),
                              void *APPptr, int addflag);
uint64_t MR_map_file_str(void *MRptr, int nmap, int nstr, char **strings, int recurse, int readflag, char *sepstr,
                         int delta, void (*mymap)(int, char *, int, void *KVptr, void *APPptr), void *APPptr);
uint64_t MR_map_file_str_add(void *MRptr, int nmap, int nstr, char **strings, int recurse, int readflag,
                             char *sepstr, int delta, void (*mymap)(int, char *, int, void *KVptr, void *APPptr),
                             void *APPptr, int addflag);
uint64_t MR_map_mr(void *MRptr, void *MRptr2,
                   void (*mymap)(uint64_t, char *, int, char *, int, void *KVptr, void *APPptr), void *APPptr);
uint64_t MR_map_mr_add(void *MRptr, void *MRptr2,
                       void (*mymap)(uint64_t, char *, int, char *, int, void *KVptr, void *APPptr), void *APPptr,
                       int addflag);

void MR_open(void *MRptr);
void MR_open_add(void *MRptr, int addflag);
void *MR_kv_open(void *MRptr); /* KVptr other MRs' callbacks add into while open */
void MR_print(void *MRptr, int proc, int nstride, int kflag, int vflag);
void MR_print_file(void *MRptr, char *file, int fflag, int proc, int nstride, int kflag, int vflag);

uint64_t MR_reduce(void *MRptr, void (*myreduce)(char *, int, char *, int, int *, void *KVptr, void *APPptr),
                   void *APPptr);
/* built-in device reducers: op = count|sum|min|max|first|last, dtype = int32|int64|float32|float64 */
uint64_t MR_reduce_builtin(void *MRptr, const char *op, const char *dtype);
/* device functors: HIP device source defining mr_map / mr_reduce (csrc/engine/devfn.h),
   compiled at run time for the GPU; a GPU MapReduce only */
uint64_t MR_map_device(void *MRptr, void *MRptr2, const char *code, int addflag);
uint64_t MR_map_device_tasks(void *MRptr, uint64_t ntask, const char *code, int addflag);
uint64_t MR_reduce_device(void *MRptr, const char *code);
uint64_t MR_compress_device(void *MRptr, const char *code);
/* stable sort by a device sort-key functor (mr_sortkey: key -> 64-bit key in the wanted order) */
uint64_t MR_sort_keys_device(void *MRptr, const char *code, int bits);
uint64_t MR_sort_values_device(void *MRptr, const char *code, int bits);
uint64_t MR_multivalue_blocks(void *MRptr, int *nblock);
void MR_multivalue_block_select(void *MRptr, int which);
int MR_multivalue_block(void *MRptr, int iblock, char **ptr_multivalue, int **ptr_valuesizes);
uint64_t MR_scan_kv(void *MRptr, void (*myscan)(char *, int, char *, int, void *), void *APPptr);
uint64_t MR_scan_kmv(void *MRptr, void (*myscan)(char *, int, char *, int, int *, void *), void *APPptr);

uint64_t MR_scrunch(void *MRptr, int numprocs, char *key, int keybytes);
uint64_t MR_sort_keys(void *MRptr, int (*mycompare)(char *, int, char *, int));
uint64_t MR_sort_keys_flag(void *MRptr, int flag);
uint64_t MR_sort_values(void *MRptr, int (*mycompare)(char *, int, char *, int));
uint64_t MR_sort_values_flag(void *MRptr, int flag);
uint64_t MR_sort_multivalues(void *MRptr, int (*mycompare)(char *, int, char *, int));
uint64_t MR_sort_multivalues_flag(void *MRptr, int flag);

/* checkpoint / restart of this rank's KV or KMV (binary SoA file per rank) */
void MR_save(void *MRptr, const char *path);
uint64_t MR_load(void *MRptr, const char *path);

uint64_t MR_kv_stats(void *MRptr, int level);
uint64_t MR_kmv_stats(void *MRptr, int level);
void MR_cummulative_stats(void *MRptr, int level, int reset);

void MR_set_mapstyle(void *MRptr, int value);
void MR_set_all2all(void *MRptr, int value);
void MR_set_verbosity(void *MRptr, int value);
void MR_set_timer(void *MRptr, int value);
void MR_set_memsize(void *MRptr, int value);
void MR_set_minpage(void *MRptr, int value);
void MR_set_maxpage(void *MRptr, int value);
void MR_set_freepage(void *MRptr, int value);
void MR_set_outofcore(void *MRptr, int value);
void MR_set_zeropage(void *MRptr, int value);
void MR_set_keyalign(void *MRptr, int value);
void MR_set_valuealign(void *MRptr, int value);
void MR_set_fpath(void *MRptr, char *str);
/* MI355X-native settings (not in the reference): shuffle receive cap per
 * round in bytes, HBM budget of the MR's data (out-of-core beyond it), pinned
 * host bytes before the spill tier writes to disk, pipelined collate (1/0) */
void MR_set_chunk_bytes(void *MRptr, int64_t value);
void MR_set_hbm_budget(void *MRptr, int64_t value);
void MR_set_host_budget(void *MRptr, int64_t value);
void MR_set_pipeline(void *MRptr, int value);

void MR_kv_add(void *KVptr, char *key, int keybytes, char *value, int valuebytes);
void MR_kv_add_multi_static(void *KVptr, int n, char *key, int keybytes, char *value, int valuebytes);
void MR_kv_add_multi_dynamic(void *KVptr, int n, char *key, int *keybytes, char *value, int *valuebytes);

/* last error message of a failed call (calls that fail print it and abort the
 * process unless MR_set_error_mode(1) was called, then they return 0/NULL) */
const char *MR_last_error(void);
void MR_set_error_mode(int return_codes);

#ifdef __cplusplus
}
#endif
#endif
