// OINK universe, MR-object registry and command I/O descriptors (reference
// oink/universe.cpp:23-99, oink/object.cpp: create_mr :96-115, copy_mr
// :123-128, permanent :135-141, input :147-231, output :237-366, cleanup
// :373-393, add_input :421-488, add_output :494-549, add_mr :560-606,
// user_input :612-671, user_output :673-712, set :714-755, expandpath
// :913-942, createdir :950-990; oink/command.cpp:21-38).
#include <cctype>
#include <cstdlib>
#include <filesystem>

#include "oink.h"

namespace mrh {
namespace oink {

namespace {
bool valid_id(const std::string& s) {
  if (s.empty()) return false;
  for (char c : s)
    if (!(std::isalnum((unsigned char)c) || c == '_')) return false;
  return true;
}
int to_int(const std::string& s, const char* what) {
  char* e = nullptr;
  long v = std::strtol(s.c_str(), &e, 10);
  if (!e || *e || s.empty()) throw Error(std::string("Illegal ") + what + " command");
  return (int)v;
}
void createdir(const std::string& path) {
  std::filesystem::path d = std::filesystem::path(path).parent_path();
  if (!d.empty()) std::filesystem::create_directories(d);
}
}  // namespace

// ====================================================================== Universe

Universe::Universe(CommPtr u, const Args& partitions, CommPtr w) : ucomm(std::move(u)) {
  me = ucomm->rank();
  nprocs = ucomm->size();
  for (auto& p : partitions) {
    size_t x = p.find('x');
    if (x != std::string::npos) {
      int n = to_int(p.substr(0, x), "-partition"), m = to_int(p.substr(x + 1), "-partition");
      for (int i = 0; i < n; ++i) sizes.push_back(m);
    } else {
      sizes.push_back(to_int(p, "-partition"));
    }
  }
  if (sizes.empty()) sizes.push_back(nprocs);
  int tot = 0;
  for (int s : sizes) tot += s;
  if (tot != nprocs) throw Error("Processor partitions are inconsistent");
  nworlds = (int)sizes.size();
  int acc = 0;
  for (int i = 0; i < nworlds; ++i) {
    if (me < acc + sizes[i]) {
      iworld = i;
      break;
    }
    acc += sizes[i];
  }
  world = nworlds == 1 ? ucomm : (w ? w : ucomm->split(iworld));
}

// ====================================================================== Object: MR registry

std::shared_ptr<MapReduce> Object::allocate_mr(int v, int t, int m, int o) {
  auto mr = std::make_shared<MapReduce>(oink_.comm);
  mr->set.verbosity = v >= 0 ? v : verbosity;
  mr->set.timer = t >= 0 ? t : timer;
  mr->set.memsize = m != 0 ? m : memsize;
  mr->set.outofcore = o >= -1 ? o : outofcore;
  mr->set.minpage = minpage;
  mr->set.maxpage = maxpage;
  mr->set.freepage = freepage;
  mr->set.zeropage = zeropage;
  if (!scratch.empty()) mr->set_fpath(scratch);
  return mr;
}

MapReduce& Object::create_mr() {
  mrs.push_back({allocate_mr(), "", false});
  return *mrs.back().mr;
}

MapReduce& Object::copy_mr(MapReduce& mr) {
  mrs.push_back({std::shared_ptr<MapReduce>(mr.copy().release()), "", false});
  return *mrs.back().mr;
}

int Object::find_mr(const std::string& name) const {
  for (size_t i = 0; i < mrs.size(); ++i)
    if (mrs[i].permanent && mrs[i].name == name) return (int)i;
  return -1;
}

bool Object::permanent(const MapReduce& mr) const {
  for (auto& e : mrs)
    if (e.mr.get() == &mr && e.permanent) return true;
  return false;
}

void Object::add_mr_named(const Args& a) {
  if (a.empty() || a.size() > 5) throw Error("Illegal mr command");
  if (!valid_id(a[0])) throw Error("MR ID must be alphanumeric or underscore characters");
  if (find_mr(a[0]) >= 0) throw Error("ID in mr command is already in use");
  int v[4] = {-1, -1, 0, -2};
  for (size_t i = 1; i < a.size(); ++i) v[i - 1] = to_int(a[i], "mr");
  mrs.push_back({allocate_mr(v[0], v[1], v[2], v[3]), a[0], true});
}

void Object::delete_mr(int index) { mrs.erase(mrs.begin() + index); }

void Object::cleanup() {
  std::vector<Entry> keep;
  for (auto& e : mrs)
    if (e.permanent) keep.push_back(e);
  mrs.swap(keep);
  inputs_.clear();
  outputs_.clear();
}

// ====================================================================== descriptors

std::string Object::expandpath(const std::string& in, const std::string& pre, bool postpend, int sub,
                               int multi) const {
  const int me = oink_.comm->rank();
  std::string p;
  if (!pre.empty() && postpend) p = pre + "/" + in + "." + std::to_string(me);
  else if (!pre.empty()) p = pre + "/" + in;
  else if (postpend) p = in + "." + std::to_string(me);
  else p = in;
  size_t k = p.find('%');
  if (k != std::string::npos) p.replace(k, 1, std::to_string(sub == 0 ? me : (me % sub) + 1));
  k = p.find('*');
  if (k != std::string::npos) p.replace(k, 1, std::to_string(multi));
  return p;
}

void Object::add_input(int index, const std::string& s) {
  InputDesc d;
  auto it = userin_.find(index);
  if (it != userin_.end()) {
    d = it->second;
    userin_.erase(it);
  }
  d.index = index;
  if ((int)inputs_.size() <= index) inputs_.resize(index + 1);
  const int imr = find_mr(s);
  if (imr >= 0) {
    d.is_mr = true;
    d.mr = mrs[imr].mr;
    inputs_[index] = d;
    return;
  }
  std::vector<std::string> items;
  if (s.rfind("v_", 0) == 0) {
    if (!oink_.variable->find(s.substr(2))) throw Error("Command input variable is unknown");
    items = oink_.variable->retrieve_all(s.substr(2));
  } else {
    items = {s};
  }
  const std::string pre = d.pflag ? d.prepend : prepend;
  const int sub = d.suflag ? d.substitute : substitute;
  for (auto& one : items)
    for (int j = 0; j < d.multi; ++j) d.strings.push_back(expandpath(one, pre, false, sub, j + 1));
  inputs_[index] = d;
}

void Object::add_output(int index, const std::string& file, const std::string& name) {
  OutputDesc d;
  auto it = userout_.find(index);
  if (it != userout_.end()) {
    d = it->second;
    userout_.erase(it);
  }
  d.index = index;
  if ((int)outputs_.size() <= index) outputs_.resize(index + 1);
  if (name != "NULL") {
    if (!valid_id(name)) throw Error("Ouptut MR ID must be alphanumeric or underscore characters");
    d.name = name;
    d.to_mr = true;
  }
  if (file != "NULL") {
    const std::string pre = d.pflag ? d.prepend : prepend;
    const int sub = d.suflag ? d.substitute : substitute;
    d.procfile = expandpath(file, pre, true, sub, 0);
    createdir(d.procfile);
    d.to_file = true;
  }
  outputs_[index] = d;
}

void Object::user_input(const Args& a) {
  if (a.size() < 3) throw Error("Illegal input command");
  const int index = to_int(a[0], "input") - 1;
  InputDesc& d = userin_[index];
  for (size_t i = 1; i < a.size(); i += 2) {
    if (i + 1 >= a.size()) throw Error("Illegal input command");
    const std::string &k = a[i], &v = a[i + 1];
    if (k == "prepend") {
      d.pflag = 1;
      d.prepend = v;
    } else if (k == "substitute") {
      d.suflag = 1;
      d.substitute = to_int(v, "input");
    } else if (k == "multi") d.multi = to_int(v, "input");
    else if (k == "mmode") d.mmode = to_int(v, "input");
    else if (k == "recurse") d.recurse = to_int(v, "input");
    else if (k == "self") d.self = to_int(v, "input");
    else if (k == "readfile") d.readfile = to_int(v, "input");
    else if (k == "nmap") d.nmap = to_int(v, "input");
    else if (k == "delta") d.delta = to_int(v, "input");
    else if (k == "sepchar") d.sepchar = v.empty() ? '\n' : v[0];
    else if (k == "sepstr") d.sepstr = v;
    else throw Error("Illegal input command");
  }
}

void Object::user_output(const Args& a) {
  if (a.size() < 3) throw Error("Illegal output command");
  const int index = to_int(a[0], "output") - 1;
  OutputDesc& d = userout_[index];
  for (size_t i = 1; i < a.size(); i += 2) {
    if (i + 1 >= a.size()) throw Error("Illegal output command");
    if (a[i] == "prepend") {
      d.pflag = 1;
      d.prepend = a[i + 1];
    } else if (a[i] == "substitute") {
      d.suflag = 1;
      d.substitute = to_int(a[i + 1], "output");
    } else {
      throw Error("Illegal output command");
    }
  }
}

void Object::set(const Args& a) {
  if (a.size() % 2) throw Error("Illegal set command");
  for (size_t i = 0; i < a.size(); i += 2) {
    const std::string &k = a[i], &v = a[i + 1];
    if (k == "scratch") scratch = v;
    else if (k == "prepend") prepend = v;
    else if (k == "verbosity") verbosity = to_int(v, "set");
    else if (k == "timer") timer = to_int(v, "set");
    else if (k == "memsize") memsize = to_int(v, "set");
    else if (k == "outofcore") outofcore = to_int(v, "set");
    else if (k == "minpage") minpage = to_int(v, "set");
    else if (k == "maxpage") maxpage = to_int(v, "set");
    else if (k == "freepage") freepage = to_int(v, "set");
    else if (k == "zeropage") zeropage = to_int(v, "set");
    else if (k == "substitute") substitute = to_int(v, "set");
    else throw Error("Illegal set command");
  }
}

MapReduce& Object::input(int index, const MapFileFn& file_fn, const MapChunkFn& chunk_fn) {
  if (index < 1 || index > (int)inputs_.size() || inputs_[index - 1].index < 0)
    throw Error("Command input invoked with invalid index");
  InputDesc& d = inputs_[index - 1];
  if (d.is_mr) return *d.mr;
  if (!file_fn && !chunk_fn) throw Error("Command input not allowed from file");
  MapReduce& mr = create_mr();
  if (d.mmode == 0) {
    if (!file_fn) throw Error("Comand input map function does not match input mode");
    mr.map_file(d.strings, d.self, d.recurse, d.readfile, file_fn);
  } else {
    if (!chunk_fn) throw Error("Command input map function does not match input mode");
    if (d.mmode == 1)
      mr.map_file_char(d.nmap, d.strings, d.self, d.recurse, d.readfile, d.sepchar, d.delta, chunk_fn);
    else
      mr.map_file_str(d.nmap, d.strings, d.self, d.recurse, d.readfile, d.sepstr, d.delta, chunk_fn);
  }
  return mr;
}

void Object::output(int index, MapReduce& mr, const Printer& pr, bool disallow_mr) {
  if (index < 1 || index > (int)outputs_.size() || outputs_[index - 1].index < 0)
    throw Error("Command output invoked with invalid index");
  OutputDesc& d = outputs_[index - 1];
  if (d.to_mr) {
    if (disallow_mr) throw Error("Command output as MR object not allowed");
    int w = -1;
    for (size_t i = 0; i < mrs.size(); ++i)
      if (mrs[i].mr.get() == &mr) w = (int)i;
    if (w < 0) throw Error("Command output called with unknown MR object");
    for (size_t i = 0; i < mrs.size(); ++i)
      if ((int)i != w && mrs[i].permanent && mrs[i].name == d.name) {
        mrs[i].permanent = false;
        mrs[i].name.clear();
      }
    mrs[w].name = d.name;
    mrs[w].permanent = true;
  }
  if (d.to_file) {
    if (!pr) throw Error("Command input not allowed to file");
    std::FILE* f = std::fopen(d.procfile.c_str(), "w");
    if (!f) throw Error("Could not open command output file " + d.procfile);
    try {
      pr(mr, f);
    } catch (...) {
      std::fclose(f);
      throw;
    }
    std::fclose(f);
  }
}

// ====================================================================== Command base

Command::Command(Oink& o)
    : oink(o), obj(*o.obj), comm(o.comm), me(o.comm->rank()), nprocs(o.comm->size()) {}

void Command::params(const Args& a) {
  if (!a.empty()) throw Error("Illegal " + name + " command");
}

void Command::inputs(const Args& a) {
  if ((int)a.size() != ninputs)
    throw Error("Illegal " + name + " command: " + std::to_string(ninputs) + " inputs required");
  for (size_t i = 0; i < a.size(); ++i) obj.add_input((int)i, a[i]);
}

void Command::outputs(const Args& a) {
  if ((int)a.size() != 2 * noutputs)
    throw Error("Illegal " + name + " command: " + std::to_string(noutputs) + " outputs (file mr) required");
  for (int i = 0; i < noutputs; ++i) obj.add_output(i, a[2 * i], a[2 * i + 1]);
}

void Command::message(const std::string& s) { oink.message(s); }

}  // namespace oink
}  // namespace mrh
