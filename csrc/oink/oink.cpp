// OINK interpreter (reference oink/oink.cpp:29-294 command line + setup,
// oink/input.cpp: file :106-183, parse :258-320, substitute :328-379,
// execute_command :386-489, built-ins :497-832).
#include "oink.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <sstream>

namespace mrh {
namespace oink {

namespace {
double now() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

std::vector<std::string> read_lines(std::istream& in) {
  std::vector<std::string> v;
  std::string l;
  while (std::getline(in, l)) v.push_back(l);
  return v;
}

// POSIX-shell-like split: whitespace separates words, '...' and "..." group
// (quotes removed), backslash escapes outside single quotes
Args shell_split(const std::string& s) {
  Args out;
  std::string cur;
  bool have = false;
  char q = 0;
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (q == '\'') {
      if (c == '\'') q = 0;
      else cur += c;
      continue;
    }
    if (q == '"') {
      if (c == '"') q = 0;
      else if (c == '\\' && i + 1 < s.size() && (s[i + 1] == '"' || s[i + 1] == '\\' || s[i + 1] == '$')) cur += s[++i];
      else cur += c;
      continue;
    }
    if (c == '\'' || c == '"') {
      q = c;
      have = true;
    } else if (c == '\\' && i + 1 < s.size()) {
      cur += s[++i];
      have = true;
    } else if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
      if (have) out.push_back(cur);
      cur.clear();
      have = false;
    } else {
      cur += c;
      have = true;
    }
  }
  if (q) throw Error("Unbalanced quotes in input line");
  if (have) out.push_back(cur);
  return out;
}
}  // namespace

std::map<std::string, CommandFactory>& command_registry() {
  static std::map<std::string, CommandFactory> r;
  return r;
}

Oink::Oink(CommPtr ucomm, const Args& partitions, Sink screen, const std::string& logfile,
           const std::vector<std::pair<std::string, Args>>& variables, const std::string& echo, CommPtr world) {
  if (!ucomm) ucomm = std::make_shared<Comm>();
  universe = std::make_unique<Universe>(ucomm, partitions, world);
  comm = universe->world;
  me = comm->rank();
  if (me == 0) screen_ = std::move(screen);
  if (me == 0 && !logfile.empty() && logfile != "none") {
    log_ = std::fopen(logfile.c_str(), "w");
    if (!log_) throw Error("Cannot open logfile " + logfile);
  }
  variable = std::make_unique<Variable>(*this);
  obj = std::make_unique<Object>(*this);
  if (!echo.empty()) b_echo({echo});
  for (auto& nv : variables) {
    Args a{nv.first, "index"};
    a.insert(a.end(), nv.second.begin(), nv.second.end());
    variable->set(a);
  }
}

Oink::~Oink() { close(); }

void Oink::close() {
  if (obj) obj->cleanup();
  if (log_) {
    std::fclose(log_);
    log_ = nullptr;
  }
}

void Oink::message(const std::string& s) {
  if (me != 0) return;
  if (screen_) screen_(s + "\n");
  if (log_) {
    std::fprintf(log_, "%s\n", s.c_str());
    std::fflush(log_);
  }
}

void Oink::emit_echo(const std::string& line) {
  if (me != 0 || label_active_) return;
  std::string l = line;
  if (l.empty() || l.back() != '\n') l += '\n';
  if (echo_screen_ && screen_) screen_(l);
  if (echo_log_ && log_) std::fputs(l.c_str(), log_);
}

// ---------------------------------------------------------------- reading

void Oink::push_file(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw Error("Cannot open input script " + path);
  files_.push_back({read_lines(in), 0, path});
}

void Oink::file(const std::string& path) {
  if (me == 0) {
    if (path.empty()) files_.push_back({read_lines(std::cin), 0, ""});
    else push_file(path);
  }
  run_files();
}

void Oink::text(const std::string& script) {
  if (me == 0) {
    std::istringstream in(script);
    files_.push_back({read_lines(in), 0, ""});
  }
  run_files();
}

bool Oink::readline(std::string& line) {
  while (!files_.empty()) {
    Src& f = files_.back();
    std::string buf;
    bool cont = false;
    while (f.pos < f.lines.size()) {
      std::string l = f.lines[f.pos++];
      size_t e = l.find_last_not_of(" \t\r");
      if (e != std::string::npos && l[e] == '&') {
        buf += l.substr(0, e) + " ";
        cont = true;
        continue;
      }
      line = buf + l;
      return true;
    }
    if (cont) {
      line = buf;
      return true;
    }
    files_.pop_back();
  }
  return false;
}

// rank 0 reads, every rank gets the line (reference input.cpp:135,148 MPI_Bcast)
void Oink::run_files() {
  while (true) {
    std::string msg;
    if (me == 0) {
      std::string line;
      msg = readline(line) ? "L" + line : std::string("E");
    }
    msg = comm->bcast(msg, 0);
    if (msg.empty() || msg[0] == 'E') {
      if (label_active_) throw Error("Label wasn't found in input script");
      break;
    }
    const std::string line = msg.substr(1);
    emit_echo(line);
    std::string cmd;
    Args args;
    parse(line, cmd, args);
    if (cmd.empty() || (label_active_ && cmd != "label")) continue;
    if (!execute(cmd, args)) throw Error("Unknown command: " + line);
  }
}

std::string Oink::one(const std::string& line) {
  emit_echo(line);
  std::string cmd;
  Args args;
  parse(line, cmd, args);
  if (cmd.empty() || (label_active_ && cmd != "label")) return "";
  if (!execute(cmd, args)) throw Error("Unknown command: " + line);
  return cmd;
}

void Oink::parse(const std::string& line, std::string& cmd, Args& args) {
  std::string s;
  char q = 0;
  for (char c : line) {  // strip comments outside quotes
    if (c == '#' && !q) break;
    if (c == q) q = 0;
    else if ((c == '"' || c == '\'') && !q) q = c;
    s += c;
  }
  if (!label_active_) s = substitute(s);
  Args t = shell_split(s);
  cmd.clear();
  args.clear();
  if (t.empty()) return;
  cmd = t[0];
  args.assign(t.begin() + 1, t.end());
}

std::string Oink::substitute(const std::string& s) {
  std::string out;
  char q = 0;
  for (size_t i = 0; i < s.size();) {
    char c = s[i];
    if (c == '$' && !q && i + 1 < s.size()) {
      std::string name;
      if (s[i + 1] == '{') {
        size_t j = s.find('}', i + 2);
        if (j == std::string::npos) throw Error("Invalid variable name");
        name = s.substr(i + 2, j - i - 2);
        i = j + 1;
      } else {
        name = s.substr(i + 1, 1);
        i += 2;
      }
      std::string v;
      if (!variable->retrieve(name, v)) throw Error("Substitution for illegal variable");
      out += v;
      continue;
    }
    if (c == q) q = 0;
    else if ((c == '"' || c == '\'') && !q) q = c;
    out += c;
    ++i;
  }
  return out;
}

// ---------------------------------------------------------------- dispatch

bool Oink::execute(const std::string& cmd, const Args& args) {
  if (cmd == "clear") b_clear(args);
  else if (cmd == "echo") b_echo(args);
  else if (cmd == "if") b_if(args);
  else if (cmd == "include") b_include(args);
  else if (cmd == "jump") b_jump(args);
  else if (cmd == "label") b_label(args);
  else if (cmd == "log") b_log(args);
  else if (cmd == "next") b_next(args);
  else if (cmd == "print") b_print(args);
  else if (cmd == "shell") b_shell(args);
  else if (cmd == "variable") variable->set(args);
  else if (cmd == "input") obj->user_input(args);
  else if (cmd == "mr") obj->add_mr_named(args);
  else if (cmd == "output") obj->user_output(args);
  else if (cmd == "set") obj->set(args);
  else {
    auto& reg = command_registry();
    auto it = reg.find(cmd);
    if (it != reg.end()) {
      std::unique_ptr<Command> c = it->second(*this);
      c->name = cmd;
      size_t i = 0;
      while (i < args.size() && args[i] != "-i" && args[i] != "-o") ++i;
      c->params(Args(args.begin(), args.begin() + i));
      bool isw = false, osw = false;
      while (i < args.size()) {
        const std::string sw = args[i];
        const std::string other = sw == "-i" ? "-o" : "-i";
        size_t j = i + 1;
        while (j < args.size() && args[j] != other) ++j;
        if (sw == "-i") {
          c->inputs(Args(args.begin() + i + 1, args.begin() + j));
          isw = true;
        } else if (sw == "-o") {
          c->outputs(Args(args.begin() + i + 1, args.begin() + j));
          osw = true;
        } else {
          throw Error("Invalid command switch");
        }
        i = j;
      }
      if (!isw) c->inputs({});
      if (!osw) c->outputs({});
      comm->barrier();
      const double t0 = now();
      try {
        c->run();
      } catch (...) {
        obj->cleanup();
        throw;
      }
      comm->barrier();
      deltatime = now() - t0;
      return true;
    }
    const int idx = obj->find_mr(cmd);
    if (idx < 0) return false;
    comm->barrier();
    const double t0 = now();
    run_mr_method(*this, idx, args);
    comm->barrier();
    deltatime = now() - t0;
  }
  return true;
}

// ---------------------------------------------------------------- built-ins

void Oink::b_clear(const Args& a) {
  if (!a.empty()) throw Error("Illegal clear command");
  obj = std::make_unique<Object>(*this);
  variable = std::make_unique<Variable>(*this);
}

void Oink::b_echo(const Args& a) {
  if (a.size() != 1 || (a[0] != "none" && a[0] != "screen" && a[0] != "log" && a[0] != "both"))
    throw Error("Illegal echo command");
  echo_screen_ = a[0] == "screen" || a[0] == "both";
  echo_log_ = a[0] == "log" || a[0] == "both";
}

// if "cond" then "cmd" ... [elif "cond" "cmd" ...] [else "cmd" ...]
void Oink::b_if(const Args& a) {
  if (a.size() < 3 || a[1] != "then") throw Error("Illegal if command");
  struct Block {
    bool has_cond;
    std::string cond;
    Args cmds;
  };
  std::vector<Block> blocks;
  std::string cur = a[0];
  bool has = true;
  size_t start = 2;
  while (true) {
    size_t j = start;
    while (j < a.size() && a[j] != "elif" && a[j] != "else") ++j;
    blocks.push_back({has, cur, Args(a.begin() + start, a.begin() + j)});
    if (j >= a.size()) break;
    if (a[j] == "elif") {
      if (j + 2 > a.size()) throw Error("Illegal if command");
      cur = a[j + 1];
      has = true;
      start = j + 2;
    } else {
      has = false;
      cur.clear();
      start = j + 1;
    }
  }
  for (auto& b : blocks) {
    const bool ok = !b.has_cond || variable->evaluate_boolean(substitute(b.cond));
    if (!ok) continue;
    if (b.cmds.empty()) throw Error("Illegal if command");
    for (auto& c : b.cmds) one(c);
    return;
  }
}

void Oink::b_include(const Args& a) {
  if (a.size() != 1) throw Error("Illegal include command");
  if (me == 0) push_file(a[0]);
}

void Oink::b_jump(const Args& a) {
  if (a.empty() || a.size() > 2) throw Error("Illegal jump command");
  if (jump_skip_) {
    jump_skip_ = 0;
    return;
  }
  if (me == 0) {
    if (files_.empty()) throw Error("jump outside of an input script");
    std::string path = a[0] == "SELF" ? files_.back().path : a[0];
    if (path.empty()) throw Error("Cannot jump SELF on stdin/text input");
    std::ifstream in(path);
    if (!in) throw Error("Cannot open input script " + path);
    files_.back() = {read_lines(in), 0, path};
  }
  if (a.size() == 2) {
    label_active_ = true;
    labelstr_ = a[1];
  }
}

void Oink::b_label(const Args& a) {
  if (a.size() != 1) throw Error("Illegal label command");
  if (label_active_ && labelstr_ == a[0]) label_active_ = false;
}

void Oink::b_log(const Args& a) {
  if (a.size() != 1) throw Error("Illegal log command");
  if (me != 0) return;
  if (log_) std::fclose(log_);
  log_ = nullptr;
  if (a[0] != "none") {
    log_ = std::fopen(a[0].c_str(), "w");
    if (!log_) throw Error("Cannot open logfile " + a[0]);
  }
}

void Oink::b_next(const Args& a) {
  if (variable->next(a)) jump_skip_ = 1;
}

void Oink::b_print(const Args& a) {
  if (a.size() != 1) throw Error("Illegal print command");
  message(substitute(a[0]));
}

void Oink::b_shell(const Args& a) {
  if (a.empty()) throw Error("Illegal shell command");
  namespace fs = std::filesystem;
  const std::string& op = a[0];
  if (op == "cd") {
    if (a.size() != 2) throw Error("Illegal shell command");
    fs::current_path(a[1]);
    return;
  }
  if (me != 0) return;
  std::error_code ec;
  if (op == "mkdir") {
    for (size_t i = 1; i < a.size(); ++i) fs::create_directories(a[i], ec);
  } else if (op == "mv") {
    if (a.size() != 3) throw Error("Illegal shell command");
    fs::rename(a[1], a[2]);
  } else if (op == "rm") {
    for (size_t i = 1; i < a.size(); ++i) fs::remove(a[i], ec);
  } else if (op == "rmdir") {
    for (size_t i = 1; i < a.size(); ++i) fs::remove(a[i], ec);
  } else {
    throw Error("Illegal shell command");
  }
}

// ---------------------------------------------------------------- command line

int main_args(CommPtr ucomm, const Args& argv) {
  std::string infile, screen_path, logfile = "log.oink", echo;
  bool screen_none = false;
  std::vector<std::pair<std::string, Args>> vars;
  Args parts;
  for (size_t i = 0; i < argv.size();) {
    const std::string& a = argv[i];
    auto need = [&](size_t k) {
      if (i + k >= argv.size()) throw Error("Invalid command-line argument");
    };
    if (a == "-in" || a == "-i") {
      need(1);
      infile = argv[i + 1];
      i += 2;
    } else if (a == "-var" || a == "-v") {
      need(2);
      size_t j = i + 2;
      while (j < argv.size() && argv[j][0] != '-') ++j;
      vars.push_back({argv[i + 1], Args(argv.begin() + i + 2, argv.begin() + j)});
      i = j;
    } else if (a == "-partition" || a == "-p") {
      size_t j = i + 1;
      while (j < argv.size() && argv[j][0] != '-') parts.push_back(argv[j++]);
      i = j;
    } else if (a == "-screen" || a == "-sc") {
      need(1);
      if (argv[i + 1] == "none") screen_none = true;
      else screen_path = argv[i + 1];
      i += 2;
    } else if (a == "-log" || a == "-l") {
      need(1);
      logfile = argv[i + 1];
      i += 2;
    } else if (a == "-echo" || a == "-e") {
      need(1);
      echo = argv[i + 1];
      i += 2;
    } else {
      throw Error("Invalid command-line argument " + a);
    }
  }
  std::shared_ptr<std::FILE> sf;
  Oink::Sink sink;
  if (!screen_none) {
    if (!screen_path.empty()) {
      sf.reset(std::fopen(screen_path.c_str(), "w"), [](std::FILE* f) {
        if (f) std::fclose(f);
      });
      if (!sf) throw Error("Cannot open screen file " + screen_path);
      sink = [sf](const std::string& s) { std::fputs(s.c_str(), sf.get()); };
    } else {
      sink = [](const std::string& s) {
        std::fputs(s.c_str(), stdout);
        std::fflush(stdout);
      };
    }
  }
  Oink o(ucomm, parts, sink, logfile, vars, echo);
  o.file(infile);
  o.close();
  return 0;
}

}  // namespace oink
}  // namespace mrh
