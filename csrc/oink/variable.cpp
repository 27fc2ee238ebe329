// OINK variables (reference oink/variable.cpp: set :98-289, next :306,
// evaluate :574-855, math_function :892-1040, keyword :1079-1090,
// evaluate_boolean :1132). Equal-style formulas use the reference precedence
// (| < & < ==,!= < <,<=,>,>= < +,- < *,/ < ^ < unary -,!), the math functions
// sqrt exp ln log sin cos tan asin acos atan atan2 random normal ceil floor
// round, the constant PI and the keywords nprocs and time.
#include <cctype>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <thread>

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
  if (!e || *e) throw Error(std::string("Illegal ") + what);
  return (int)v;
}
int prec(const std::string& op) {
  if (op == "|") return 1;
  if (op == "&") return 2;
  if (op == "==" || op == "!=") return 3;
  if (op == "<" || op == "<=" || op == ">" || op == ">=") return 4;
  if (op == "+" || op == "-") return 5;
  if (op == "*" || op == "/") return 6;
  if (op == "^") return 7;
  return 8;  // NEG, !
}
enum Tok { NUM = 0, PAREN = 1, WORD = 2, OP = 3 };

std::vector<std::pair<int, std::string>> tokenize(const std::string& s) {
  std::vector<std::pair<int, std::string>> t;
  size_t i = 0, n = s.size();
  while (i < n) {
    char c = s[i];
    if (std::isspace((unsigned char)c)) {
      ++i;
    } else if (c == '(') {
      int depth = 1;
      size_t j = i + 1;
      while (j < n && depth) {
        if (s[j] == '(') ++depth;
        else if (s[j] == ')') --depth;
        ++j;
      }
      if (depth) throw Error("Invalid syntax in variable formula");
      t.emplace_back(PAREN, s.substr(i + 1, j - i - 2));
      i = j;
    } else if (std::isdigit((unsigned char)c) || c == '.') {
      size_t j = i;
      while (j < n && (std::isdigit((unsigned char)s[j]) || s[j] == '.')) ++j;
      if (j < n && (s[j] == 'e' || s[j] == 'E')) {
        ++j;
        if (j < n && (s[j] == '+' || s[j] == '-')) ++j;
        while (j < n && std::isdigit((unsigned char)s[j])) ++j;
      }
      t.emplace_back(NUM, s.substr(i, j - i));
      i = j;
    } else if (std::isalpha((unsigned char)c)) {
      size_t j = i;
      while (j < n && (std::isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
      t.emplace_back(WORD, s.substr(i, j - i));
      i = j;
    } else {
      std::string two = s.substr(i, 2);
      if (two == "==" || two == "!=" || two == "<=" || two == ">=") {
        t.emplace_back(OP, two);
        i += 2;
      } else if (two == "&&" || two == "||") {
        t.emplace_back(OP, two.substr(0, 1));
        i += 2;
      } else if (std::string("+-*/^<>!&|").find(c) != std::string::npos) {
        t.emplace_back(OP, std::string(1, c));
        ++i;
      } else if (c == '=') {
        t.emplace_back(OP, "==");
        ++i;
      } else {
        throw Error("Invalid syntax in variable formula");
      }
    }
  }
  return t;
}

std::vector<std::string> split_args(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  int depth = 0;
  for (char c : s) {
    if (c == ',' && depth == 0) {
      out.push_back(cur);
      cur.clear();
      continue;
    }
    if (c == '(') ++depth;
    if (c == ')') --depth;
    cur += c;
  }
  out.push_back(cur);
  return out;
}
}  // namespace

void Variable::set(const Args& a) {
  if (a.size() < 2) throw Error("Illegal variable command");
  const std::string& name = a[0];
  const std::string& style = a[1];
  if (!valid_id(name)) throw Error("Variable name must be alphanumeric or underscore characters");
  if (style == "delete") {
    vars_.erase(name);
    return;
  }
  if ((style == "index" || style == "loop" || style == "world" || style == "universe" || style == "uloop") &&
      vars_.count(name))
    return;
  const Universe& uni = *oink_.universe;
  Var v;
  v.style = style;
  if (style == "index") {
    if (a.size() < 3) throw Error("Illegal variable command");
    v.data.assign(a.begin() + 2, a.end());
  } else if (style == "loop") {
    Args rest(a.begin() + 2, a.end());
    bool pad = false;
    if (!rest.empty() && rest.back() == "pad") {
      rest.pop_back();
      pad = true;
    }
    int first, last;
    if (rest.size() == 1) {
      first = 1;
      last = to_int(rest[0], "variable command");
    } else if (rest.size() == 2) {
      first = to_int(rest[0], "variable command");
      last = to_int(rest[1], "variable command");
    } else {
      throw Error("Illegal variable command");
    }
    if (last <= 0 || first > last) throw Error("Illegal variable command");
    v.data.assign((size_t)(last - first + 1), std::string());
    v.offset = first;
    v.pad = pad ? (int)std::to_string(last).size() : 0;
  } else if (style == "world") {
    if ((int)a.size() - 2 != uni.nworlds) throw Error("World variable count doesn't match # of partitions");
    v.data.assign(a.begin() + 2, a.end());
    v.which = uni.iworld;
  } else if (style == "universe" || style == "uloop") {
    if (style == "universe") {
      v.data.assign(a.begin() + 2, a.end());
    } else {
      if (a.size() < 3) throw Error("Illegal variable command");
      int n = to_int(a[2], "variable command");
      v.data.assign((size_t)n, std::string());
      v.pad = (a.size() == 4 && a[3] == "pad") ? (int)std::to_string(n).size() : 0;
      v.offset = 1;
    }
    if ((int)v.data.size() < uni.nworlds) throw Error("Universe/uloop variable count < # of partitions");
    v.which = uni.iworld;
    if (uni.me == 0) {
      std::FILE* f = std::fopen("tmp.oink.variable", "w");
      if (!f) throw Error("Cannot open temporary file for world counter");
      std::fprintf(f, "%d\n", uni.nworlds);
      std::fclose(f);
    }
  } else if (style == "string" || style == "equal") {
    if (a.size() != 3) throw Error("Illegal variable command");
    auto it = vars_.find(name);
    if (it != vars_.end() && it->second.style != style) throw Error("Cannot redefine variable as a different style");
    v.data = {a[2]};
  } else {
    throw Error("Illegal variable command");
  }
  vars_[name] = v;
}

bool Variable::next(const Args& names) {
  if (names.empty()) throw Error("Illegal next command");
  for (auto& n : names)
    if (!vars_.count(n)) throw Error("Invalid variable in next command");
  const std::string style = vars_[names[0]].style;
  if (style == "string" || style == "equal" || style == "world")
    throw Error("Invalid variable style with next command");
  bool flag = false;
  if (style == "index" || style == "loop") {
    for (auto& n : names) {
      Var& v = vars_[n];
      if (++v.which >= (int)v.data.size()) {
        flag = true;
        vars_.erase(n);
      }
    }
    return flag;
  }
  // universe / uloop: next unused value from a shared counter file (reference
  // variable.cpp:340-370: rename-based lock between worlds)
  const Universe& uni = *oink_.universe;
  int nxt = 0;
  const int world_me = uni.world ? uni.world->rank() : 0;
  if (world_me == 0) {
    while (std::rename("tmp.oink.variable", "tmp.oink.variable.lock") != 0)
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    {
      std::ifstream in("tmp.oink.variable.lock");
      in >> nxt;
    }
    std::FILE* f = std::fopen("tmp.oink.variable.lock", "w");
    std::fprintf(f, "%d\n", nxt + 1);
    std::fclose(f);
    std::rename("tmp.oink.variable.lock", "tmp.oink.variable");
  }
  nxt = std::atoi(oink_.comm->bcast(std::to_string(nxt), 0).c_str());
  for (auto& n : names) {
    Var& v = vars_[n];
    v.which = nxt;
    if (v.which >= (int)v.data.size()) {
      flag = true;
      vars_.erase(n);
    }
  }
  return flag;
}

bool Variable::retrieve(const std::string& n, std::string& out) {
  auto it = vars_.find(n);
  if (it == vars_.end() || it->second.which >= (int)it->second.data.size()) return false;
  const Var& v = it->second;
  if (v.style == "index" || v.style == "world" || v.style == "universe" || v.style == "string") {
    out = v.data[v.which];
  } else if (v.style == "loop" || v.style == "uloop") {
    std::string s = std::to_string(v.which + v.offset);
    if (v.pad && (int)s.size() < v.pad) s = std::string(v.pad - s.size(), '0') + s;
    out = s;
  } else {
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%.10g", evaluate(v.data[0]));
    out = buf;
  }
  return true;
}

std::vector<std::string> Variable::retrieve_all(const std::string& n) {
  auto it = vars_.find(n);
  if (it == vars_.end()) throw Error("Command input variable is unknown");
  const Var& v = it->second;
  if (v.style == "equal") throw Error("Command input is equal-style variable");
  if (v.style == "loop" || v.style == "uloop") {
    std::vector<std::string> o;
    for (size_t i = 0; i < v.data.size(); ++i) o.push_back(std::to_string((int)i + v.offset));
    return o;
  }
  return v.data;
}

double Variable::uniform() {
  // splitmix64
  uint64_t z = (rng_state_ += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

double Variable::math(const std::string& w, const std::vector<double>& a) {
  auto need = [&](size_t k) {
    if (a.size() != k) throw Error("Invalid math function in variable formula");
  };
  if (w == "random" || w == "normal") {
    need(3);
    if (!rng_init_) {
      if (a[2] <= 0) throw Error("Invalid math function in variable formula");
      rng_state_ = (uint64_t)a[2];
      rng_init_ = true;
    }
    if (w == "random") return uniform() * (a[1] - a[0]) + a[0];
    double u1 = std::max(uniform(), 1e-300), u2 = uniform();
    return a[0] + a[1] * std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
  if (w == "atan2") {
    need(2);
    return std::atan2(a[0], a[1]);
  }
  need(1);
  const double x = a[0];
  if ((w == "sqrt" && x < 0) || ((w == "ln" || w == "log") && x <= 0) ||
      ((w == "asin" || w == "acos") && std::fabs(x) > 1))
    throw Error("Invalid math function in variable formula");
  if (w == "sqrt") return std::sqrt(x);
  if (w == "exp") return std::exp(x);
  if (w == "ln") return std::log(x);
  if (w == "log") return std::log10(x);
  if (w == "sin") return std::sin(x);
  if (w == "cos") return std::cos(x);
  if (w == "tan") return std::tan(x);
  if (w == "asin") return std::asin(x);
  if (w == "acos") return std::acos(x);
  if (w == "atan") return std::atan(x);
  if (w == "ceil") return std::ceil(x);
  if (w == "floor") return std::floor(x);
  if (w == "round") return (x - std::floor(x) >= 0.5) ? std::ceil(x) : std::floor(x);
  throw Error("Invalid math function in variable formula");
}

double Variable::word(const std::string& w, const std::vector<std::pair<int, std::string>>& toks, size_t& pos) {
  if (w.rfind("v_", 0) == 0) {
    std::string val;
    if (!retrieve(w.substr(2), val)) throw Error("Invalid variable evaluation in variable formula");
    return std::strtod(val.c_str(), nullptr);
  }
  if (pos < toks.size() && toks[pos].first == PAREN) {
    std::vector<double> args;
    for (auto& s : split_args(toks[pos].second)) args.push_back(evaluate(s));
    ++pos;
    return math(w, args);
  }
  if (w == "PI") return M_PI;
  if (w == "nprocs") return (double)oink_.comm->size();
  if (w == "time") return oink_.deltatime;
  throw Error("Invalid math/group/special function in variable formula");
}

double Variable::evaluate(const std::string& s) {
  auto toks = tokenize(s);
  size_t pos = 0;
  std::vector<double> args;
  std::vector<std::string> ops;
  auto apply = [&](const std::string& op) {
    if (args.empty()) throw Error("Invalid syntax in variable formula");
    double b = args.back();
    args.pop_back();
    if (op == "NEG") {
      args.push_back(-b);
      return;
    }
    if (op == "!") {
      args.push_back(b == 0.0 ? 1.0 : 0.0);
      return;
    }
    if (args.empty()) throw Error("Invalid syntax in variable formula");
    double a = args.back();
    args.pop_back();
    double r;
    if (op == "+") r = a + b;
    else if (op == "-") r = a - b;
    else if (op == "*") r = a * b;
    else if (op == "/") {
      if (b == 0.0) throw Error("Divide by 0 in variable formula");
      r = a / b;
    } else if (op == "^") {
      if (a == 0.0 && b == 0.0) throw Error("Power by 0 in variable formula");
      r = std::pow(a, b);
    } else if (op == "==") r = a == b;
    else if (op == "!=") r = a != b;
    else if (op == "<") r = a < b;
    else if (op == "<=") r = a <= b;
    else if (op == ">") r = a > b;
    else if (op == ">=") r = a >= b;
    else if (op == "&") r = (a != 0 && b != 0);
    else r = (a != 0 || b != 0);
    args.push_back(r);
  };
  bool expect_arg = true;
  while (true) {
    if (pos >= toks.size()) {
      if (expect_arg) throw Error("Invalid syntax in variable formula");
      while (!ops.empty()) {
        apply(ops.back());
        ops.pop_back();
      }
      break;
    }
    auto [kind, val] = toks[pos++];
    if (kind != OP) {
      if (!expect_arg) throw Error("Invalid syntax in variable formula");
      expect_arg = false;
      if (kind == NUM) args.push_back(std::strtod(val.c_str(), nullptr));
      else if (kind == PAREN) args.push_back(evaluate(val));
      else args.push_back(word(val, toks, pos));
      continue;
    }
    if (expect_arg) {
      if (val == "-") {
        ops.push_back("NEG");
        continue;
      }
      if (val == "!") {
        ops.push_back("!");
        continue;
      }
      throw Error("Invalid syntax in variable formula");
    }
    while (!ops.empty() && prec(ops.back()) >= prec(val)) {
      apply(ops.back());
      ops.pop_back();
    }
    ops.push_back(val);
    expect_arg = true;
  }
  if (args.size() != 1) throw Error("Invalid syntax in variable formula");
  return args[0];
}

// if-command conditions: numbers compare numerically, other words as strings
bool Variable::evaluate_boolean(const std::string& s) {
  static const char* ops[] = {"==", "!=", "<=", ">=", "<", ">"};
  for (const char* op : ops) {
    size_t p = s.find(op);
    if (p == std::string::npos) continue;
    auto trim = [](std::string x) {
      size_t a = x.find_first_not_of(" \t"), b = x.find_last_not_of(" \t");
      return a == std::string::npos ? std::string() : x.substr(a, b - a + 1);
    };
    std::string a = trim(s.substr(0, p)), b = trim(s.substr(p + std::strlen(op)));
    char *ea = nullptr, *eb = nullptr;
    double x = std::strtod(a.c_str(), &ea), y = std::strtod(b.c_str(), &eb);
    const bool num = !a.empty() && !b.empty() && ea && !*ea && eb && !*eb;
    const std::string o(op);
    if (num) {
      if (o == "==") return x == y;
      if (o == "!=") return x != y;
      if (o == "<=") return x <= y;
      if (o == ">=") return x >= y;
      if (o == "<") return x < y;
      return x > y;
    }
    if (o == "==") return a == b;
    if (o == "!=") return a != b;
    if (o == "<=") return a <= b;
    if (o == ">=") return a >= b;
    if (o == "<") return a < b;
    return a > b;
  }
  return evaluate(s) != 0.0;
}

}  // namespace oink
}  // namespace mrh
