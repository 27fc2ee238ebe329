// OINK named-callback library (see callbacks.h). Reference parity:
// map_read_edge.cpp:14-25 (and the label/weight/vertex variants),
// map_read_words.cpp:14-30, map_edge_to_vertices.cpp:14-20, map_invert.cpp:11-15,
// map_edge_upper, map_add_label / map_add_weight, reduce_count.cpp:13-20,
// reduce_cull.cpp:12-20, scan_print_edge.cpp:10-16 and friends.
#include "callbacks.h"

#include <cinttypes>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <vector>

#include "oink.h"
#include "kernels/launch.h"

#include <ATen/hip/HIPContext.h>

namespace mrh {
namespace oink {

namespace {
at::TensorOptions opt(at::Device d, at::ScalarType t) { return at::TensorOptions().device(d).dtype(t); }

inline bool ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// whitespace tokens of [s, s+n)
template <typename F>
void tokens(const char* s, size_t n, F&& f) {
  size_t i = 0;
  while (i < n) {
    while (i < n && (ws(s[i]) || s[i] == 0)) ++i;
    if (i >= n) break;
    size_t j = i;
    while (j < n && !ws(s[j]) && s[j] != 0) ++j;
    f(s + i, j - i);
    i = j;
  }
}

uint64_t tok_u64(const char* p, size_t len) {
  char buf[32];
  len = std::min<size_t>(len, sizeof(buf) - 1);
  std::memcpy(buf, p, len);
  buf[len] = 0;
  return std::strtoull(buf, nullptr, 10);
}
double tok_f64(const char* p, size_t len) {
  char buf[64];
  len = std::min<size_t>(len, sizeof(buf) - 1);
  std::memcpy(buf, p, len);
  buf[len] = 0;
  return std::strtod(buf, nullptr);
}

// k columns per row; col types: 'u' u64, 'i' int32, 'd' double
struct Cols {
  std::vector<std::vector<uint64_t>> u;
  std::vector<std::vector<double>> d;
  std::vector<std::vector<int32_t>> i;
  int64_t n = 0;
};
Cols read_cols(const char* s, size_t n, const char* types) {
  const int k = (int)std::strlen(types);
  std::vector<std::pair<const char*, size_t>> t;
  tokens(s, n, [&](const char* p, size_t len) { t.emplace_back(p, len); });
  Cols c;
  c.n = (int64_t)t.size() / k;
  c.u.resize(k);
  c.d.resize(k);
  c.i.resize(k);
  for (int64_t r = 0; r < c.n; ++r)
    for (int j = 0; j < k; ++j) {
      const auto& tk = t[(size_t)r * k + j];
      if (types[j] == 'u') c.u[j].push_back(tok_u64(tk.first, tk.second));
      else if (types[j] == 'i') c.i[j].push_back((int32_t)std::strtol(std::string(tk.first, tk.second).c_str(), nullptr, 10));
      else c.d[j].push_back(tok_f64(tk.first, tk.second));
    }
  return c;
}

template <typename T>
at::Tensor host_tensor(const std::vector<T>& v, at::ScalarType st) {
  at::Tensor t = at::empty({(int64_t)v.size()}, at::TensorOptions().dtype(st));
  if (!v.empty()) std::memcpy(t.data_ptr(), v.data(), v.size() * sizeof(T));
  return t;
}
at::Tensor u64t(const std::vector<uint64_t>& v) { return host_tensor(v, at::kLong); }

std::string host_bytes(const at::Tensor& t) {
  at::Tensor h = t.to(at::kCPU).contiguous();
  return std::string((const char*)h.data_ptr(), (size_t)h.numel() * h.element_size());
}

void out_str(std::FILE* f, const std::string& s) {
  if (!s.empty()) std::fwrite(s.data(), 1, s.size(), f);
  MapReduce::wsize += (int64_t)s.size();
}
}  // namespace

void add_tensors(KeyValue& kv, const at::Tensor& keys, const at::Tensor& vals, const at::Tensor& voff) {
  const int64_t n = keys.dim() ? keys.size(0) : 1;
  if (n == 0) return;
  const at::Device dev = kv.device();
  at::Tensor kd = keys.contiguous().view(at::kByte).reshape({-1});
  at::Tensor vd = vals.defined() ? vals.contiguous().view(at::kByte).reshape({-1}) : at::empty({0}, opt(dev, at::kByte));
  c10::optional<at::Tensor> vo;
  if (voff.defined()) vo = voff;
  kv.add_kv(make_kv(kd, c10::nullopt, vd, vo, n, dev));
}

at::Tensor edges_of(const KV& kv) { return kv.kdata.view(at::kLong).view({-1, 2}); }
at::Tensor u64_col(const at::Tensor& data) { return data.view(at::kLong); }

// ====================================================================== file parsers

void parse_edge(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "uu");
  add_tensors(kv, at::stack({u64t(c.u[0]), u64t(c.u[1])}, 1));
}
void parse_edge_label(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "uui");
  add_tensors(kv, at::stack({u64t(c.u[0]), u64t(c.u[1])}, 1), host_tensor(c.i[2], at::kInt));
}
void parse_edge_weight(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "uud");
  add_tensors(kv, at::stack({u64t(c.u[0]), u64t(c.u[1])}, 1), host_tensor(c.d[2], at::kDouble));
}
void parse_vertex_label(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "ui");
  add_tensors(kv, u64t(c.u[0]), host_tensor(c.i[1], at::kInt));
}
void parse_vertex_weight(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "ud");
  add_tensors(kv, u64t(c.u[0]), host_tensor(c.d[1], at::kDouble));
}
void parse_vertex_vertex(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "uu");
  add_tensors(kv, u64t(c.u[0]), u64t(c.u[1]));
}
void parse_tri(const char* s, size_t n, KeyValue& kv) {
  Cols c = read_cols(s, n, "uuu");
  add_tensors(kv, at::stack({u64t(c.u[0]), u64t(c.u[1]), u64t(c.u[2])}, 1));
}
// "v n1 n2 ..." lines -> one (v, ni) pair per neighbour
void parse_neighbors(const char* s, size_t n, KeyValue& kv) {
  std::vector<uint64_t> ks, vs;
  size_t a = 0;
  while (a < n) {
    size_t b = a;
    while (b < n && s[b] != '\n') ++b;
    std::vector<uint64_t> row;
    tokens(s + a, b - a, [&](const char* p, size_t len) { row.push_back(tok_u64(p, len)); });
    for (size_t j = 1; j < row.size(); ++j) {
      ks.push_back(row[0]);
      vs.push_back(row[j]);
    }
    a = b + 1;
  }
  add_tensors(kv, u64t(ks), u64t(vs));
}
// words (strtok " \t\n\f\r"), key = word + NUL, tokenised on the device by the
// same kernel as wordfreq
void parse_words(const char* s, size_t n, KeyValue& kv) {
  const at::Device dev = kv.device();
  at::Tensor t = at::zeros({(int64_t)n + 64}, at::TensorOptions().dtype(at::kByte));
  if (n) std::memcpy(t.data_ptr(), s, n);
  kv.add_kv(map_words(t.to(dev), (int64_t)n));
}

const std::map<std::string, Parser>& file_parsers() {
  static const std::map<std::string, Parser> m = {
      {"read_edge", parse_edge},
      {"read_edge_label", parse_edge_label},
      {"read_edge_weight", parse_edge_weight},
      {"read_vertex_label", parse_vertex_label},
      {"read_vertex_weight", parse_vertex_weight},
      {"read_vertex_vertex", parse_vertex_vertex},
      {"read_words", parse_words},
      {"read_neighbors", parse_neighbors},
      {"read_tri", parse_tri},
  };
  return m;
}

MapFileFn file_reader(Parser p, int64_t* nfiles) {
  return [p, nfiles](int, const char* fname, KeyValue& kv) {
    std::ifstream in(fname, std::ios::binary);
    if (!in) throw Error(std::string("Could not open file ") + fname);
    std::stringstream ss;
    ss << in.rdbuf();
    std::string data = ss.str();
    MapReduce::rsize += (int64_t)data.size();
    if (nfiles) ++*nfiles;
    p(data.c_str(), data.size(), kv);
  };
}

MapChunkFn chunk_reader(Parser p) {
  return [p](int, char* str, int size, KeyValue& kv) { p(str, (size_t)size, kv); };
}

// ====================================================================== map/mr batch callbacks

void edge_to_vertex(const KV& src, KeyValue& kv) {
  if (src.n) add_tensors(kv, edges_of(src).select(1, 0).contiguous());
}
void edge_to_vertices(const KV& src, KeyValue& kv) {
  if (!src.n) return;
  at::Tensor e = edges_of(src);
  add_tensors(kv, at::cat({e.select(1, 0), e.select(1, 1)}));
}
void edge_to_vertex_pair(const KV& src, KeyValue& kv) {
  if (!src.n) return;
  at::Tensor e = edges_of(src);
  add_tensors(kv, e.select(1, 0).contiguous(), e.select(1, 1).contiguous());
}
// vi < vj, self loops dropped (vertex ids < 2^63)
void edge_upper(const KV& src, KeyValue& kv) {
  if (!src.n) return;
  at::Tensor e = edges_of(src);
  if (e.is_cuda() && e.is_contiguous()) {  // flags, the engine's scan, one write kernel (util.hip)
    const hipStream_t s = at::hip::getCurrentHIPStream();
    at::Tensor flag = at::empty({src.n}, opt(e.device(), at::kInt));
    k::edge_ne_flags(e.data_ptr<int64_t>(), src.n, reinterpret_cast<uint32_t*>(flag.data_ptr<int32_t>()), s);
    at::Tensor pos = scan_u32(flag);  // u32 [n + 1]
    uint32_t m = 0;
    read_small(s, {{reinterpret_cast<const uint32_t*>(pos.data_ptr()) + src.n, &m, 4}});
    at::Tensor out = at::empty({(int64_t)m, 2}, opt(e.device(), at::kLong));
    k::edge_upper_write(e.data_ptr<int64_t>(), src.n, reinterpret_cast<const uint32_t*>(pos.data_ptr()),
                        out.data_ptr<int64_t>(), s);
    add_tensors(kv, out);
    return;
  }
  at::Tensor a = e.select(1, 0), b = e.select(1, 1);
  at::Tensor keep = a != b;
  at::Tensor lo = at::minimum(a, b).index({keep}), hi = at::maximum(a, b).index({keep});
  add_tensors(kv, at::stack({lo, hi}, 1));
}
void invert(const KV& src, KeyValue& kv) {
  KV o;
  o.n = src.n;
  o.kw = src.vw;
  o.vw = src.kw;
  o.kdata = src.vdata;
  o.vdata = src.kdata;
  if (src.vw < 0) o.koff = src.voff;
  if (src.kw < 0) o.voff = src.koff;
  kv.add_kv(o);
}
void add_label(const KV& src, KeyValue& kv) {
  KV o = src;
  o.vw = 4;
  o.voff = at::Tensor();
  o.vdata = at::ones({src.n}, opt(src.device(), at::kInt)).view(at::kByte);
  kv.add_kv(o);
}
void add_weight(const KV& src, KeyValue& kv) {
  KV o = src;
  o.vw = 8;
  o.voff = at::Tensor();
  o.vdata = at::ones({src.n}, opt(src.device(), at::kDouble)).view(at::kByte);
  kv.add_kv(o);
}

const std::map<std::string, MapBatchFn>& mr_maps() {
  static const std::map<std::string, MapBatchFn> m = {
      {"edge_to_vertex", edge_to_vertex}, {"edge_to_vertices", edge_to_vertices},
      {"edge_to_vertex_pair", edge_to_vertex_pair}, {"edge_upper", edge_upper},
      {"invert", invert}, {"add_label", add_label}, {"add_weight", add_weight},
  };
  return m;
}

const std::map<std::string, std::string>& reduces() {
  static const std::map<std::string, std::string> m = {{"count", "count"}, {"cull", "first"}};
  return m;
}

// ====================================================================== scans / hashes / compares

const std::map<std::string, ScanKVFn>& scans() {
  static const std::map<std::string, ScanKVFn> m = {
      {"print_edge",
       [](char* k, int, char*, int) {
         uint64_t e[2];
         std::memcpy(e, k, 16);
         std::printf("%" PRIu64 " %" PRIu64 "\n", e[0], e[1]);
       }},
      {"print_vertex",
       [](char* k, int, char*, int) {
         uint64_t v;
         std::memcpy(&v, k, 8);
         std::printf("%" PRIu64 "\n", v);
       }},
      {"print_string_int",
       [](char* k, int kb, char* v, int) {
         int32_t c;
         std::memcpy(&c, v, 4);
         std::printf("%s %d\n", std::string(k, strnlen(k, (size_t)kb)).c_str(), c);
       }},
  };
  return m;
}

const std::map<std::string, HashFn>& hashes() {
  static const std::map<std::string, HashFn> m = {
      {"hash_vertex",
       [](char* k, int) {
         uint64_t v;
         std::memcpy(&v, k, 8);
         return (int)(v & 0x7fffffffu);
       }},
  };
  return m;
}

const std::map<std::string, CompareFn>& compares() {
  static const std::map<std::string, CompareFn> m = {
      {"compare_uint64",
       [](char* a, int, char* b, int) {
         uint64_t x, y;
         std::memcpy(&x, a, 8);
         std::memcpy(&y, b, 8);
         return (x > y) - (x < y);
       }},
  };
  return m;
}

// ====================================================================== printers

namespace {
struct HostKV {
  std::string k, v;
  at::Tensor koff, voff;
  int64_t n = 0;
  int kw = 0, vw = 0;
  const char* key(int64_t i) const { return k.data() + (kw >= 0 ? i * kw : koff.data_ptr<int64_t>()[i]); }
  int64_t klen(int64_t i) const { return kw >= 0 ? kw : koff.data_ptr<int64_t>()[i + 1] - koff.data_ptr<int64_t>()[i]; }
  const char* val(int64_t i) const { return v.data() + (vw >= 0 ? i * vw : voff.data_ptr<int64_t>()[i]); }
  int64_t vlen(int64_t i) const { return vw >= 0 ? vw : voff.data_ptr<int64_t>()[i + 1] - voff.data_ptr<int64_t>()[i]; }
};
HostKV host_kv(MapReduce& mr) {
  mr.flatten();
  if (!mr.kv) throw Error("Command output requires KeyValue pairs");
  const KV& kv = *mr.kv;
  HostKV h;
  h.n = kv.n;
  h.kw = kv.kw;
  h.vw = kv.vw;
  h.k = host_bytes(kv.kdata);
  h.v = host_bytes(kv.vdata);
  if (kv.kw < 0) h.koff = kv.koff.to(at::kCPU).contiguous();
  if (kv.vw < 0) h.voff = kv.voff.to(at::kCPU).contiguous();
  return h;
}
template <typename T>
T rd(const char* p) {
  T x;
  std::memcpy(&x, p, sizeof(T));
  return x;
}
char* put_u64(char* p, uint64_t x) {
  char tmp[24];
  int n = 0;
  do {
    tmp[n++] = (char)('0' + x % 10);
    x /= 10;
  } while (x);
  while (n) *p++ = tmp[--n];
  return p;
}
// rows of u64 columns as decimal text, written in blocks
void write_u64_rows(std::FILE* f, const uint64_t* d, int64_t n, int ncol) {
  std::string buf;
  buf.resize(1 << 20);
  char* p = &buf[0];
  std::string all;
  for (int64_t i = 0; i < n; ++i) {
    if (p - &buf[0] > (1 << 20) - 128) {
      out_str(f, std::string(&buf[0], p));
      p = &buf[0];
    }
    for (int c = 0; c < ncol; ++c) {
      p = put_u64(p, d[i * ncol + c]);
      *p++ = c + 1 < ncol ? ' ' : '\n';
    }
  }
  out_str(f, std::string(&buf[0], p));
}
}  // namespace

void print_edge(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  write_u64_rows(f, reinterpret_cast<const uint64_t*>(h.k.data()), h.n, 2);
}
void print_vertex(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  write_u64_rows(f, reinterpret_cast<const uint64_t*>(h.k.data()), h.n, 1);
}
void print_tri(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  write_u64_rows(f, reinterpret_cast<const uint64_t*>(h.k.data()), h.n, 3);
}
void print_vertex_u64(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  char line[64];
  for (int64_t i = 0; i < h.n; ++i) {
    std::snprintf(line, sizeof(line), "%" PRIu64 " %" PRIu64 "\n", rd<uint64_t>(h.key(i)), rd<uint64_t>(h.val(i)));
    s += line;
  }
  out_str(f, s);
}
void print_string_int(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  for (int64_t i = 0; i < h.n; ++i) {
    const char* k = h.key(i);
    s.append(k, strnlen(k, (size_t)h.klen(i)));
    s += ' ';
    s += std::to_string(rd<int32_t>(h.val(i)));
    s += '\n';
  }
  out_str(f, s);
}
void print_vertex_int(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  char line[64];
  for (int64_t i = 0; i < h.n; ++i) {
    std::snprintf(line, sizeof(line), "%" PRIu64 " %d\n", rd<uint64_t>(h.key(i)), rd<int32_t>(h.val(i)));
    s += line;
  }
  out_str(f, s);
}
void print_vertex_double(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  char line[64];
  for (int64_t i = 0; i < h.n; ++i) {
    std::snprintf(line, sizeof(line), "%" PRIu64 " %g\n", rd<uint64_t>(h.key(i)), rd<double>(h.val(i)));
    s += line;
  }
  out_str(f, s);
}
void print_edge_weight(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  char line[96];
  for (int64_t i = 0; i < h.n; ++i) {
    std::snprintf(line, sizeof(line), "%" PRIu64 " %" PRIu64 " %g\n", rd<uint64_t>(h.key(i)),
                  rd<uint64_t>(h.key(i) + 8), rd<double>(h.val(i)));
    s += line;
  }
  out_str(f, s);
}
void print_neighbors(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  for (int64_t i = 0; i < h.n; ++i) {
    s += std::to_string(rd<uint64_t>(h.key(i)));
    const int64_t nb = h.vlen(i) / 8;
    for (int64_t j = 0; j < nb; ++j) {
      s += ' ';
      s += std::to_string(rd<uint64_t>(h.val(i) + 8 * j));
    }
    s += '\n';
  }
  out_str(f, s);
}
// "v distance source"
void print_sssp(MapReduce& mr, std::FILE* f) {
  HostKV h = host_kv(mr);
  std::string s;
  char line[96];
  for (int64_t i = 0; i < h.n; ++i) {
    std::snprintf(line, sizeof(line), "%" PRIu64 " %g %" PRId64 "\n", rd<uint64_t>(h.key(i)), rd<double>(h.val(i)),
                  rd<int64_t>(h.val(i) + 8));
    s += line;
  }
  out_str(f, s);
}

}  // namespace oink
}  // namespace mrh
