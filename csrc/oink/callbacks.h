// OINK named-callback library (reference oink/map_*.cpp, reduce_*.cpp,
// scan_*.cpp; types oink/typedefs.h: VERTEX = uint64, EDGE = {u64 vi, vj},
// LABEL = int, WEIGHT = double).
//
// File readers parse text on the host and append one device batch per file;
// map/mr callbacks run on the whole device KV at once (ATen ops + engine
// kernels on the MI355X); reduces are the engine's built-in segmented-reduce
// kernels; printers stream a device KV to a text file.
#pragma once
#include <ATen/ATen.h>

#include <cstdio>
#include <functional>
#include <map>
#include <string>

#include "engine/keyvalue.h"
#include "engine/mapreduce.h"

namespace mrh {
namespace oink {

// append n rows: fixed-width keys/values are [n, ...] tensors of any dtype
// (one row per pair); vals undefined = NULL values; voff = variable values
void add_tensors(KeyValue& kv, const at::Tensor& keys, const at::Tensor& vals = at::Tensor(),
                 const at::Tensor& voff = at::Tensor());
// EDGE keys of a KV as [n,2] int64 (device view)
at::Tensor edges_of(const KV& kv);
// u64 keys / values as int64 views
at::Tensor u64_col(const at::Tensor& data);

// ------------------------------------------------------------------ file readers (map/file)
// text parsers over a buffer (shared by whole-file and chunked input)
void parse_edge(const char* s, size_t n, KeyValue& kv);
void parse_edge_label(const char* s, size_t n, KeyValue& kv);
void parse_edge_weight(const char* s, size_t n, KeyValue& kv);
void parse_vertex_label(const char* s, size_t n, KeyValue& kv);
void parse_vertex_weight(const char* s, size_t n, KeyValue& kv);
void parse_vertex_vertex(const char* s, size_t n, KeyValue& kv);
void parse_words(const char* s, size_t n, KeyValue& kv);
void parse_neighbors(const char* s, size_t n, KeyValue& kv);
void parse_tri(const char* s, size_t n, KeyValue& kv);

using Parser = void (*)(const char*, size_t, KeyValue&);
const std::map<std::string, Parser>& file_parsers();
// whole-file and chunk adapters of a parser
MapFileFn file_reader(Parser p, int64_t* nfiles = nullptr);
MapChunkFn chunk_reader(Parser p);

// ------------------------------------------------------------------ map/mr batch callbacks
void edge_to_vertex(const KV& src, KeyValue& kv);
void edge_to_vertices(const KV& src, KeyValue& kv);
void edge_to_vertex_pair(const KV& src, KeyValue& kv);
void edge_upper(const KV& src, KeyValue& kv);
void invert(const KV& src, KeyValue& kv);
void add_label(const KV& src, KeyValue& kv);
void add_weight(const KV& src, KeyValue& kv);
const std::map<std::string, MapBatchFn>& mr_maps();

// ------------------------------------------------------------------ reduces: name -> builtin device reducer
const std::map<std::string, std::string>& reduces();  // count -> count, cull -> first

// ------------------------------------------------------------------ scans / hashes / compares (scripts)
const std::map<std::string, ScanKVFn>& scans();
const std::map<std::string, HashFn>& hashes();
const std::map<std::string, CompareFn>& compares();

// ------------------------------------------------------------------ printers (MR -> per-rank text file)
void print_edge(MapReduce& mr, std::FILE* f);
void print_vertex(MapReduce& mr, std::FILE* f);
void print_string_int(MapReduce& mr, std::FILE* f);
void print_vertex_int(MapReduce& mr, std::FILE* f);
void print_vertex_u64(MapReduce& mr, std::FILE* f);
void print_vertex_double(MapReduce& mr, std::FILE* f);
void print_edge_weight(MapReduce& mr, std::FILE* f);
void print_neighbors(MapReduce& mr, std::FILE* f);
void print_tri(MapReduce& mr, std::FILE* f);
void print_sssp(MapReduce& mr, std::FILE* f);

}  // namespace oink
}  // namespace mrh
