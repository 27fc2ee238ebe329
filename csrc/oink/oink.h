// OINK: the MapReduce scripting layer, native C++ on the MI355X engine.
//
// Same script language and command set as the reference's OINK
// (oink/oink.cpp, input.cpp, variable.cpp, object.cpp, mrmpi.cpp,
// universe.cpp, command.cpp and the named commands/callbacks): rank 0 reads
// lines (`&` continuation) and broadcasts them; `#` comments; `$x` / `${name}`
// substitution; quoted arguments; built-ins (clear echo if include jump label
// log next print shell variable input mr output set); named commands with
// `-i` / `-o` descriptors; `<mrname> <method> args` drives any MapReduce
// method on a named MR. Commands and callbacks are registered in static
// tables (commands.cpp, callbacks.cpp) — no code-generation step (the
// reference's Make.py / style_*.h).
//
// Every named command keeps the reference's inputs/outputs/params contract;
// the data path underneath is the device engine (HBM-resident KV/KMV, HIP
// kernels, RCCL shuffles), and the iterative graph commands run on the
// native plans of csrc/engine/graphplan.h.
#pragma once
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "engine/comm.h"
#include "engine/mapreduce.h"

namespace mrh {
namespace oink {

using Args = std::vector<std::string>;

struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

class Oink;

// -partition NxM ...: the universe split into worlds (reference oink/universe.cpp)
class Universe {
 public:
  // world: this rank's world communicator when the caller already split the
  // universe (host engines split through torch.distributed); else split here
  Universe(CommPtr ucomm, const Args& partitions, CommPtr world = nullptr);
  CommPtr ucomm, world;
  int me = 0, nprocs = 1, nworlds = 1, iworld = 0;
  std::vector<int> sizes;
};

// Variables (reference oink/variable.cpp): styles index, loop, world,
// universe, uloop, string, equal; `next`; equal-style formula evaluator
class Variable {
 public:
  explicit Variable(Oink& o) : oink_(o) {}
  void set(const Args& a);
  // returns true when a variable ran past its last value (jump is skipped)
  bool next(const Args& names);
  bool find(const std::string& n) const { return vars_.count(n) > 0; }
  // nullptr-like: ok=false when undefined / exhausted
  bool retrieve(const std::string& n, std::string& out);
  std::vector<std::string> retrieve_all(const std::string& n);
  double evaluate(const std::string& s);
  bool evaluate_boolean(const std::string& s);

 private:
  struct Var {
    std::string style;
    std::vector<std::string> data;
    int which = 0, offset = 0, pad = 0;
  };
  double word(const std::string& w, const std::vector<std::pair<int, std::string>>& toks, size_t& pos);
  double math(const std::string& f, const std::vector<double>& a);
  Oink& oink_;
  std::map<std::string, Var> vars_;
  bool rng_init_ = false;
  uint64_t rng_state_ = 0;
  double uniform();
};

// per-command input / output descriptors (reference oink/object.cpp)
struct InputDesc {
  int index = -1;
  std::string prepend;
  int pflag = 0, suflag = 0, substitute = 0, multi = 1, mmode = 0, recurse = 0, self = 0, readfile = 0, nmap = 0,
      delta = 80;
  char sepchar = '\n';
  std::string sepstr = "\n";
  bool is_mr = false;
  std::shared_ptr<MapReduce> mr;
  std::vector<std::string> strings;
};
struct OutputDesc {
  int index = -1;
  std::string name, prepend, procfile;
  int pflag = 0, suflag = 0, substitute = 0;
  bool to_mr = false, to_file = false;
};

using Printer = std::function<void(MapReduce&, std::FILE*)>;

// Registry of named (permanent) and temporary MR objects + the I/O
// descriptors of the command being run
class Object {
 public:
  explicit Object(Oink& o) : oink_(o) {}
  struct Entry {
    std::shared_ptr<MapReduce> mr;
    std::string name;
    bool permanent = false;
  };
  std::vector<Entry> mrs;

  std::shared_ptr<MapReduce> allocate_mr(int verbosity = -1, int timer = -1, int memsize = 0, int outofcore = -2);
  MapReduce& create_mr();
  MapReduce& copy_mr(MapReduce& mr);
  int find_mr(const std::string& name) const;
  bool permanent(const MapReduce& mr) const;
  void add_mr_named(const Args& a);  // `mr ID [verbosity timer memsize outofcore]`
  void delete_mr(int index);
  void cleanup();                     // drop temporaries + descriptors after a command

  void add_input(int index, const std::string& s);
  void add_output(int index, const std::string& file, const std::string& name);
  void user_input(const Args& a);
  void user_output(const Args& a);
  void set(const Args& a);

  // MR for input #index (1-based): the named MR itself, or a new temporary MR
  // filled from the descriptor's files (mmode 0: whole files -> file_fn,
  // 1/2: chunks split on sepchar / sepstr -> chunk_fn)
  MapReduce& input(int index, const MapFileFn& file_fn = nullptr, const MapChunkFn& chunk_fn = nullptr);
  // name `mr` (if -o ... name) and/or write it to the per-rank file via `pr`
  void output(int index, MapReduce& mr, const Printer& pr = nullptr, bool disallow_mr = false);

  std::string expandpath(const std::string& in, const std::string& prepend, bool postpend, int substitute,
                         int multi) const;

  // global settings (`set` command)
  int verbosity = 0, timer = 0, memsize = 64, outofcore = 0, minpage = 0, maxpage = 0, freepage = 1, zeropage = 0,
      substitute = 0;
  std::string scratch, prepend;

 private:
  Oink& oink_;
  std::vector<InputDesc> inputs_;
  std::vector<OutputDesc> outputs_;
  std::map<int, InputDesc> userin_;
  std::map<int, OutputDesc> userout_;
};

// named-command plugin base (reference oink/command.h:16-28)
class Command {
 public:
  explicit Command(Oink& o);
  virtual ~Command() = default;
  virtual void params(const Args& a);
  virtual void inputs(const Args& a);
  virtual void outputs(const Args& a);
  virtual void run() = 0;
  std::string name;
  int ninputs = 0, noutputs = 0;

 protected:
  void message(const std::string& s);
  Oink& oink;
  Object& obj;
  CommPtr comm;
  int me, nprocs;
};

using CommandFactory = std::function<std::unique_ptr<Command>(Oink&)>;
std::map<std::string, CommandFactory>& command_registry();

class Oink {
 public:
  using Sink = std::function<void(const std::string&)>;
  // ucomm: the universe; partitions: "-partition" specs; screen: rank-0 screen
  // output (nullptr = none); logfile: "none" or a path
  Oink(CommPtr ucomm, const Args& partitions = {}, Sink screen = nullptr, const std::string& logfile = "log.oink",
       const std::vector<std::pair<std::string, Args>>& variables = {}, const std::string& echo = "",
       CommPtr world = nullptr);
  ~Oink();

  // run a script: a file path, or stdin when path is empty
  void file(const std::string& path);
  // run script text
  void text(const std::string& script);
  // one command line; returns the command name ("" for blank/comment lines)
  std::string one(const std::string& line);
  void close();

  void message(const std::string& s);  // rank 0: screen + log
  std::string substitute(const std::string& s);

  std::unique_ptr<Universe> universe;
  CommPtr comm;  // this world
  int me = 0;
  std::unique_ptr<Variable> variable;
  std::unique_ptr<Object> obj;
  double deltatime = 0.0;

 private:
  struct Src {
    std::vector<std::string> lines;
    size_t pos = 0;
    std::string path;
  };
  void run_files();
  bool readline(std::string& line);
  void parse(const std::string& line, std::string& cmd, Args& args);
  bool execute(const std::string& cmd, const Args& args);
  void emit_echo(const std::string& line);
  void push_file(const std::string& path);
  // built-ins
  void b_clear(const Args& a);
  void b_echo(const Args& a);
  void b_if(const Args& a);
  void b_include(const Args& a);
  void b_jump(const Args& a);
  void b_label(const Args& a);
  void b_log(const Args& a);
  void b_next(const Args& a);
  void b_print(const Args& a);
  void b_shell(const Args& a);

  Sink screen_;
  std::FILE* log_ = nullptr;
  int echo_screen_ = 0, echo_log_ = 1;
  bool label_active_ = false;
  std::string labelstr_;
  int jump_skip_ = 0;
  std::vector<Src> files_;
};

// script-level MapReduce method call `<mrname> <method> args` (reference oink/mrmpi.cpp)
void run_mr_method(Oink& o, int index, const Args& a);

// command line: oink [-in file] [-var name v ...] [-partition NxM ...]
// [-screen file|none] [-log file|none] [-echo style]; returns exit status
int main_args(CommPtr ucomm, const Args& argv);

}  // namespace oink
}  // namespace mrh
