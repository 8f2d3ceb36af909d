// JSON-schema constrained decoding engine -- see grammar.h.
#include "grammar.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <stdexcept>

namespace vwa {

// ============================================================================ tiny JSON reader
namespace {

struct JVal {
  enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  double n = 0;
  bool b = false;
  std::string s;
  std::vector<JVal> a;
  std::vector<std::pair<std::string, JVal>> o;
  const JVal* get(const std::string& k) const {
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JParser {
  const std::string& s;
  size_t i = 0;
  explicit JParser(const std::string& str) : s(str) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  }
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("grammar IR: ") + m); }
  JVal parse() {
    ws();
    if (i >= s.size()) fail("eof");
    JVal v;
    char c = s[i];
    if (c == '{') {
      v.t = JVal::OBJ;
      ++i;
      ws();
      if (s[i] == '}') { ++i; return v; }
      while (true) {
        ws();
        JVal k = parse();
        if (k.t != JVal::STR) fail("key");
        ws();
        if (s[i++] != ':') fail(":");
        v.o.emplace_back(k.s, parse());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == '}') { ++i; break; }
        fail("obj");
      }
    } else if (c == '[') {
      v.t = JVal::ARR;
      ++i;
      ws();
      if (s[i] == ']') { ++i; return v; }
      while (true) {
        v.a.push_back(parse());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == ']') { ++i; break; }
        fail("arr");
      }
    } else if (c == '"') {
      v.t = JVal::STR;
      ++i;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\') {
          ++i;
          char e = s[i];
          if (e == 'n') v.s += '\n';
          else if (e == 't') v.s += '\t';
          else if (e == 'u') {
            unsigned cp = std::stoul(s.substr(i + 1, 4), nullptr, 16);
            v.s += (char)cp;
            i += 4;
          } else v.s += e;
          ++i;
        } else v.s += s[i++];
      }
      ++i;
    } else if (c == 't') { v.t = JVal::BOOL; v.b = true; i += 4; }
    else if (c == 'f') { v.t = JVal::BOOL; v.b = false; i += 5; }
    else if (c == 'n') { v.t = JVal::NUL; i += 4; }
    else {
      v.t = JVal::NUM;
      size_t j = i;
      while (j < s.size() && (isdigit((unsigned char)s[j]) || s[j] == '-' || s[j] == '+' || s[j] == '.' || s[j] == 'e' || s[j] == 'E')) ++j;
      v.n = std::stod(s.substr(i, j - i));
      i = j;
    }
    return v;
  }
};

enum { O_OPEN = 0, O_KEYQ, O_KEY, O_COLON, O_VAL, O_AFTER };
enum { R_OPEN = 0, R_KEYQ, R_KEY, R_COLON, R_VAL, R_AFTER };
enum { A_OPEN = 0, A_VAL, A_AFTER, A_COMMA };

inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

// Digits so far spell the magnitude `mag` (`count` digits, sign `neg`): can appending k >= 0
// more digits (none after a leading zero, at most 15 in all) give a value in [lo, hi]?
inline bool int_completable(double mag, int count, bool neg, double lo, double hi) {
  const double mlo = neg ? std::max(0.0, -hi) : std::max(0.0, lo);
  const double mhi = neg ? -lo : hi;
  if (mhi < mlo) return false;
  const int kmax = (mag == 0 && count >= 1) ? 0 : 15 - count;
  double scale = 1.0;
  for (int k = 0; k <= kmax; ++k, scale *= 10.0) {
    const double a = mag * scale, b = a + scale - 1.0;  // values reachable with k more digits
    if (a > mhi) return false;
    if (b >= mlo) return true;
  }
  return false;
}
inline bool printable(unsigned char c) { return c >= 0x20 && c <= 0x7e; }
inline void set_first(Node& n, unsigned char c) { n.first[c >> 3] |= (uint8_t)(1u << (c & 7)); }
inline bool has_first(const Node& n, unsigned char c) { return (n.first[c >> 3] >> (c & 7)) & 1u; }

int digits_of(double v) {
  long long a = (long long)std::fabs(v);
  int d = 1;
  while (a >= 10) { a /= 10; ++d; }
  return d;
}

}  // namespace

// ============================================================================ Grammar
Grammar::Grammar(const std::string& ir_json) {
  JParser p(ir_json);
  JVal root = p.parse();
  const JVal* nodes = root.get("nodes");
  if (!nodes || nodes->t != JVal::ARR) throw std::runtime_error("grammar IR: nodes missing");
  root_ = root.get("root") ? (int)root.get("root")->n : 0;
  auto num = [](const JVal& o, const char* k, double d) {
    const JVal* v = o.get(k);
    return v ? v->n : d;
  };
  for (const JVal& jn : nodes->a) {
    Node n;
    const std::string& t = jn.get("t")->s;
    if (t == "obj") {
      n.kind = N_OBJ;
      for (const JVal& pr : jn.get("props")->a) n.props.push_back(Prop{pr.a[0].s, (int)pr.a[1].n, pr.a[2].b});
    } else if (t == "rec") {
      n.kind = N_REC;
      n.item = (int)num(jn, "v", 0);
      n.max_items = (int)num(jn, "max", 4);
      n.key_max = (int)num(jn, "klen", 24);
    } else if (t == "arr") {
      n.kind = N_ARR;
      n.item = (int)num(jn, "item", 0);
      n.min_items = (int)num(jn, "min", 0);
      n.max_items = (int)num(jn, "max", 8);
    } else if (t == "str") {
      n.kind = N_STR;
      n.max_len = (int)num(jn, "max", 64);
    } else if (t == "enum") {
      n.kind = N_ENUM;
      for (const JVal& v : jn.get("vals")->a) n.values.push_back(v.s);
    } else if (t == "const") {
      n.kind = N_CONST;
      n.values.push_back(jn.get("s")->s);
    } else if (t == "int") {
      n.kind = N_INT;
      n.lo = num(jn, "min", 0);
      n.hi = num(jn, "max", 1e9);
    } else if (t == "num") {
      n.kind = N_NUM;
      n.lo = num(jn, "min", 0);
      n.hi = num(jn, "max", 1);
      n.frac = (int)num(jn, "frac", 3);
    } else if (t == "bool") {
      n.kind = N_BOOL;
    } else if (t == "null") {
      n.kind = N_NULL;
    } else if (t == "alt") {
      n.kind = N_ALT;
      for (const JVal& v : jn.get("opts")->a) n.opts.push_back((int)v.n);
    } else {
      throw std::runtime_error("grammar IR: unknown node type " + t);
    }
    nodes_.push_back(std::move(n));
  }
  for (Node& n : nodes_) {
    if (n.kind == N_CONST) n.lit = lit_id(n.values[0]);
  }
  lit_true_ = lit_id("true");
  lit_false_ = lit_id("false");
  lit_null_ = lit_id("null");
  finalize();
}

int Grammar::lit_id(const std::string& s) {
  for (size_t i = 0; i < lits_.size(); ++i)
    if (lits_[i] == s) return (int)i;
  lits_.push_back(s);
  return (int)lits_.size() - 1;
}

int Grammar::node_min_len(int i, std::vector<int>& visiting) {
  Node& n = nodes_[i];
  if (visiting[i] == 2) return n.min_len;
  if (visiting[i] == 1) return 1 << 20;  // recursion without a base case: treat as huge
  visiting[i] = 1;
  int m = 0;
  switch (n.kind) {
    case N_OBJ: {
      int cnt = 0;
      for (const Prop& p : n.props)
        if (p.required) {
          m += (int)p.key.size() + 3 + node_min_len(p.node, visiting);
          ++cnt;
        }
      m += std::max(0, cnt - 1) + 2;
      break;
    }
    case N_REC: node_min_len(n.item, visiting); m = 2; break;
    case N_ARR: {
      int ml = node_min_len(n.item, visiting);
      m = 2 + n.min_items * ml + std::max(0, n.min_items - 1);
      break;
    }
    case N_STR: m = 2; break;
    case N_ENUM: {
      m = 1 << 20;
      for (auto& v : n.values) m = std::min(m, (int)v.size() + 2);
      break;
    }
    case N_CONST: m = (int)n.values[0].size(); break;
    case N_INT: m = (n.lo <= 0 && n.hi >= 0) ? 1 : digits_of(std::min(std::fabs(n.lo), std::fabs(n.hi))) + (n.hi < 0 ? 1 : 0); break;
    case N_NUM: m = 1; break;
    case N_BOOL: m = 4; break;
    case N_NULL: m = 4; break;
    case N_ALT: {
      m = 1 << 20;
      for (int o : n.opts) m = std::min(m, node_min_len(o, visiting));
      break;
    }
  }
  n.min_len = m;
  visiting[i] = 2;
  return m;
}

void Grammar::compute_first(int i, std::vector<int>& visiting) {
  Node& n = nodes_[i];
  if (visiting[i]) return;
  visiting[i] = 1;
  switch (n.kind) {
    case N_OBJ: case N_REC: set_first(n, '{'); break;
    case N_ARR: set_first(n, '['); break;
    case N_STR: case N_ENUM: set_first(n, '"'); break;
    case N_CONST: set_first(n, (unsigned char)n.values[0][0]); break;
    case N_INT: case N_NUM:
      for (char c = '0'; c <= '9'; ++c) set_first(n, (unsigned char)c);
      if (n.lo < 0) set_first(n, '-');
      break;
    case N_BOOL: set_first(n, 't'); set_first(n, 'f'); break;
    case N_NULL: set_first(n, 'n'); break;
    case N_ALT:
      for (int o : n.opts) {
        compute_first(o, visiting);
        for (int b = 0; b < 32; ++b) n.first[b] |= nodes_[o].first[b];
      }
      break;
  }
}

void Grammar::finalize() {
  std::vector<int> vis(nodes_.size(), 0);
  for (int i = 0; i < (int)nodes_.size(); ++i) node_min_len(i, vis);
  std::vector<int> vis2(nodes_.size(), 0);
  for (int i = 0; i < (int)nodes_.size(); ++i) compute_first(i, vis2);
  for (Node& n : nodes_) {
    if (n.kind != N_OBJ) continue;
    const int P = (int)n.props.size();
    n.rest_after.assign(P + 2, 0);
    // rest_after[j+1] = sum over required k >= j+1 of (1 + keylen + 3 + min_len)  (index shifted by one)
    for (int k = P - 1; k >= 0; --k) {
      const Prop& p = n.props[k];
      n.rest_after[k] = n.rest_after[k + 1] + (p.required ? 1 + (int)p.key.size() + 3 + nodes_[p.node].min_len : 0);
    }
  }
}

State Grammar::initial() const {
  State s;
  s.depth = 1;
  s.used = 0;
  s.done = false;
  std::memset(&s.st[0], 0, sizeof(Frame));
  s.st[0].kind = F_VALUE;
  s.st[0].node = (int16_t)root_;
  return s;
}

void Grammar::pop(State& s) const {
  s.depth--;
  if (s.depth == 0) {
    s.done = true;
    return;
  }
  Frame& p = s.st[s.depth - 1];
  switch (p.kind) {
    case F_OBJ: if (p.phase == O_VAL) p.phase = O_AFTER; break;
    case F_REC:
      if (p.phase == R_KEY) p.phase = R_COLON;
      else if (p.phase == R_VAL) { p.phase = R_AFTER; p.count++; }
      break;
    case F_ARR: if (p.phase == A_VAL) { p.phase = A_AFTER; p.count++; } break;
    default: break;
  }
}

static inline Frame& push_frame(State& s, uint8_t kind, int node) {
  Frame& f = s.st[s.depth++];
  std::memset(&f, 0, sizeof(Frame));
  f.kind = kind;
  f.node = (int16_t)node;
  return f;
}

bool Grammar::push_value(State& s, int node, unsigned char c) const {
  const Node& n = nodes_[node];
  if (!has_first(n, c)) return false;
  if (s.depth >= kMaxDepth - 1) return false;
  switch (n.kind) {
    case N_OBJ: { Frame& f = push_frame(s, F_OBJ, node); f.phase = O_OPEN; f.idx = 0; return true; }
    case N_REC: { Frame& f = push_frame(s, F_REC, node); f.phase = R_OPEN; return true; }
    case N_ARR: { Frame& f = push_frame(s, F_ARR, node); f.phase = A_OPEN; return true; }
    case N_STR: { Frame& f = push_frame(s, F_STR, node); f.aux = n.max_len; return true; }
    case N_ENUM: { push_frame(s, F_ENUM, node); return true; }
    case N_CONST: case N_BOOL: case N_NULL: {
      const int id = n.kind == N_CONST ? n.lit : (n.kind == N_NULL ? lit_null_ : (c == 't' ? lit_true_ : lit_false_));
      Frame& f = push_frame(s, F_LIT, node);
      f.aux = id;
      f.idx = 1;
      if ((size_t)f.idx == lits_[id].size()) pop(s);
      return true;
    }
    case N_INT: { push_frame(s, F_INT, node); return feed(s, c); }
    case N_NUM: { push_frame(s, F_NUM, node); return feed(s, c); }
    case N_ALT:
      for (int o : n.opts)
        if (has_first(nodes_[o], c)) return push_value(s, o, c);
      return false;
  }
  return false;
}

bool Grammar::feed(State& s, unsigned char c) const {
  while (true) {
    if (s.depth == 0) return false;
    Frame& f = s.st[s.depth - 1];
    switch (f.kind) {
      case F_VALUE: {
        const int node = f.node;
        s.depth--;
        return push_value(s, node, c);
      }
      case F_OBJ: {
        const Node& n = nodes_[f.node];
        const int P = (int)n.props.size();
        auto last_cand = [&](int from) {
          int r = from;
          while (r < P && !n.props[r].required) ++r;
          return std::min(r, P - 1);
        };
        switch (f.phase) {
          case O_OPEN:
            if (c == '"' && f.idx < P) { f.phase = O_KEY; f.blen = 0; return true; }
            if (c == '}' && n.rest_after[f.idx] == 0) { pop(s); return true; }
            return false;
          case O_KEYQ:
            if (c == '"') { f.phase = O_KEY; f.blen = 0; return true; }
            return false;
          case O_KEY: {
            const int hi = last_cand(f.idx);
            if (c == '"') {
              for (int j = f.idx; j <= hi; ++j) {
                const std::string& k = n.props[j].key;
                if ((int)k.size() == f.blen && std::memcmp(k.data(), f.buf, f.blen) == 0) {
                  f.idx = (int16_t)j;
                  f.phase = O_COLON;
                  return true;
                }
              }
              return false;
            }
            if (f.blen >= kBuf) return false;
            for (int j = f.idx; j <= hi; ++j) {
              const std::string& k = n.props[j].key;
              if ((int)k.size() > f.blen && (unsigned char)k[f.blen] == c && std::memcmp(k.data(), f.buf, f.blen) == 0) {
                f.buf[f.blen++] = (char)c;
                return true;
              }
            }
            return false;
          }
          case O_COLON:
            if (c != ':') return false;
            if (s.depth >= kMaxDepth - 1) return false;
            f.phase = O_VAL;
            { Frame& v = push_frame(s, F_VALUE, n.props[f.idx].node); (void)v; }
            return true;
          case O_AFTER:
            if (c == ',' && f.idx + 1 < P) { f.idx = (int16_t)(f.idx + 1); f.phase = O_KEYQ; return true; }
            if (c == '}' && n.rest_after[f.idx + 1] == 0) { pop(s); return true; }
            return false;
          default: return false;  // O_VAL: child should be on top
        }
      }
      case F_REC: {
        const Node& n = nodes_[f.node];
        switch (f.phase) {
          case R_OPEN:
            if (c == '"' && f.count < n.max_items) {
              f.phase = R_KEY;
              Frame& k = push_frame(s, F_STR, -1);
              k.aux = n.key_max;
              return true;
            }
            if (c == '}') { pop(s); return true; }
            return false;
          case R_KEYQ:
            if (c == '"') {
              f.phase = R_KEY;
              Frame& k = push_frame(s, F_STR, -1);
              k.aux = n.key_max;
              return true;
            }
            return false;
          case R_COLON:
            if (c != ':') return false;
            f.phase = R_VAL;
            push_frame(s, F_VALUE, n.item);
            return true;
          case R_AFTER:
            if (c == ',' && f.count < n.max_items) { f.phase = R_KEYQ; return true; }
            if (c == '}') { pop(s); return true; }
            return false;
          default: return false;
        }
      }
      case F_ARR: {
        const Node& n = nodes_[f.node];
        switch (f.phase) {
          case A_OPEN:
            if (c == ']' && n.min_items == 0) { pop(s); return true; }
            if (n.max_items == 0) return false;
            f.phase = A_VAL;
            return push_value(s, n.item, c);
          case A_COMMA:
            f.phase = A_VAL;
            return push_value(s, n.item, c);
          case A_AFTER:
            if (c == ',' && f.count < n.max_items) { f.phase = A_COMMA; return true; }
            if (c == ']' && f.count >= n.min_items) { pop(s); return true; }
            return false;
          default: return false;
        }
      }
      case F_STR: {
        if (f.flag) {
          if (c == '"' || c == '\\') { f.flag = 0; f.count++; return true; }
          return false;
        }
        if (c == '"') { pop(s); return true; }
        if (c == '\\') {
          if (f.count + 2 > f.aux) return false;
          f.flag = 1;
          f.count++;
          return true;
        }
        if (printable(c) && f.count + 1 <= f.aux) { f.count++; return true; }
        return false;
      }
      case F_ENUM: {
        const Node& n = nodes_[f.node];
        if (c == '"') {
          for (const std::string& v : n.values)
            if ((int)v.size() == f.blen && std::memcmp(v.data(), f.buf, f.blen) == 0) { pop(s); return true; }
          return false;
        }
        if (f.blen >= kBuf) return false;
        for (const std::string& v : n.values)
          if ((int)v.size() > f.blen && (unsigned char)v[f.blen] == c && std::memcmp(v.data(), f.buf, f.blen) == 0) {
            f.buf[f.blen++] = (char)c;
            return true;
          }
        return false;
      }
      case F_LIT: {
        const std::string& t = lits_[f.aux];
        if ((unsigned char)t[f.idx] != c) return false;
        f.idx++;
        if ((size_t)f.idx == t.size()) pop(s);
        return true;
      }
      case F_INT: {
        const Node& n = nodes_[f.node];
        const bool neg = f.flag & 1;
        if (c == '-' && f.count == 0 && !neg && n.lo < 0) { f.flag |= 1; return true; }
        if (is_digit(c) && !(f.count == 1 && f.val == 0) && f.count < 15) {
          const double nv = f.val * 10 + (c - '0');
          // admissible only if some completion of the digits lands in [lo, hi]: a "0" for a
          // positive integer (timeout_ms >= 1) would otherwise be a dead end -- no digit may
          // follow a leading zero and 0 itself is out of range
          if (int_completable(nv, f.count + 1, neg, n.lo, n.hi)) { f.val = nv; f.count++; return true; }
        }
        // not a continuation: terminate the number if complete and re-feed c to the parent
        if (f.count >= 1) {
          const double v = neg ? -f.val : f.val;
          if (v >= n.lo && v <= n.hi) { pop(s); continue; }
        }
        return false;
      }
      case F_NUM: {
        const Node& n = nodes_[f.node];
        const bool neg = f.flag & 1, infrac = f.flag & 2;
        const double maxabs = neg ? -n.lo : n.hi;
        if (c == '-' && f.count == 0 && !neg && !infrac && n.lo < 0) { f.flag |= 1; return true; }
        if (is_digit(c)) {
          if (!infrac) {
            if (!(f.count == 1 && f.val == 0) && f.count < 12) {
              const double nv = f.val * 10 + (c - '0');
              if (nv <= maxabs) { f.val = nv; f.count++; return true; }
            }
          } else if (f.aux < n.frac) {
            const double nv = f.val + (c - '0') * std::pow(10.0, -(f.aux + 1));
            if (nv <= maxabs + 1e-12) { f.val = nv; f.aux++; return true; }
          }
        }
        if (c == '.' && !infrac && f.count >= 1 && n.frac > 0 && f.val < maxabs) { f.flag |= 2; return true; }
        if (f.count >= 1 && (!infrac || f.aux >= 1)) {
          const double v = neg ? -f.val : f.val;
          if (v >= n.lo - 1e-12 && v <= n.hi + 1e-12) { pop(s); continue; }
        }
        return false;
      }
    }
    return false;
  }
}

bool Grammar::step(State& s, unsigned char c) const {
  if (s.done) return false;
  if (!feed(s, c)) return false;
  s.used++;
  return true;
}

int Grammar::frame_remaining(const Frame& f) const {
  switch (f.kind) {
    case F_VALUE: return nodes_[f.node].min_len;
    case F_OBJ: {
      const Node& n = nodes_[f.node];
      const int P = (int)n.props.size();
      switch (f.phase) {
        case O_OPEN: return (n.rest_after[f.idx] > 0 ? n.rest_after[f.idx] - 1 : 0) + 1;
        case O_KEYQ: case O_KEY: {
          int best = 1 << 20;
          int r = f.idx;
          while (r < P && !n.props[r].required) ++r;
          r = std::min(r, P - 1);
          for (int j = f.idx; j <= r; ++j) {
            const Prop& p = n.props[j];
            if (f.phase == O_KEY) {
              if ((int)p.key.size() < f.blen || std::memcmp(p.key.data(), f.buf, f.blen) != 0) continue;
              best = std::min(best, (int)p.key.size() - f.blen + 2 + nodes_[p.node].min_len + n.rest_after[j + 1]);
            } else {
              best = std::min(best, (int)p.key.size() + 3 + nodes_[p.node].min_len + n.rest_after[j + 1]);
            }
          }
          return best + 1;
        }
        case O_COLON: return 1 + nodes_[n.props[f.idx].node].min_len + n.rest_after[f.idx + 1] + 1;
        case O_VAL: case O_AFTER: return n.rest_after[f.idx + 1] + 1;
      }
      return 0;
    }
    case F_REC: {
      const Node& n = nodes_[f.node];
      switch (f.phase) {
        case R_OPEN: return 1;
        case R_KEYQ: return 3 + nodes_[n.item].min_len + 1;
        case R_KEY: return 1 + nodes_[n.item].min_len + 1;
        case R_COLON: return 1 + nodes_[n.item].min_len + 1;
        default: return 1;
      }
    }
    case F_ARR: {
      const Node& n = nodes_[f.node];
      const int ml = nodes_[n.item].min_len;
      switch (f.phase) {
        case A_OPEN: return (n.min_items > 0 ? n.min_items * ml + (n.min_items - 1) : 0) + 1;
        case A_COMMA: { const int r = std::max(1, n.min_items - (int)f.count); return r * ml + (r - 1) + 1; }
        case A_VAL: { const int r = std::max(0, n.min_items - (int)f.count - 1); return r * (ml + 1) + 1; }
        default: { const int r = std::max(0, n.min_items - (int)f.count); return r * (ml + 1) + 1; }
      }
    }
    case F_STR: return 1 + f.flag;
    case F_ENUM: {
      const Node& n = nodes_[f.node];
      int best = 1 << 20;
      for (const std::string& v : n.values)
        if ((int)v.size() >= f.blen && std::memcmp(v.data(), f.buf, f.blen) == 0) best = std::min(best, (int)v.size() - f.blen);
      return best + 1;
    }
    case F_LIT: return (int)lits_[f.aux].size() - f.idx;
    case F_INT: {
      const Node& n = nodes_[f.node];
      if (f.count == 0) return 1;
      const double v = (f.flag & 1) ? -f.val : f.val;
      return (v >= n.lo && v <= n.hi) ? 0 : 1;
    }
    case F_NUM: {
      if (f.count == 0) return 1;
      if ((f.flag & 2) && f.aux == 0) return 1;
      return 0;
    }
  }
  return 0;
}

int Grammar::min_completion(const State& s) const {
  if (s.done) return 0;
  int r = 0;
  for (int i = 0; i < s.depth; ++i) r += frame_remaining(s.st[i]);
  return r;
}

std::string Grammar::canon(const State& s) const {
  std::string k;
  k.reserve(16 + s.depth * 24);
  k.push_back((char)s.done);
  for (int i = 0; i < s.depth; ++i) {
    const Frame& f = s.st[i];
    k.push_back((char)f.kind);
    k.push_back((char)f.phase);
    k.append(reinterpret_cast<const char*>(&f.node), 2);
    k.append(reinterpret_cast<const char*>(&f.idx), 2);
    switch (f.kind) {
      case F_STR: {
        const int rem = std::min(f.aux - f.count, 255);
        k.push_back((char)rem);
        k.push_back((char)f.flag);
        break;
      }
      case F_OBJ: case F_ENUM:
        k.push_back((char)f.blen);
        k.append(f.buf, f.blen);
        break;
      case F_REC: case F_ARR: {
        // The item count only matters near the bounds: below min_items (closing not yet
        // allowed) and within reach of max_items (whether ',' may follow the current item).  One
        // token spans at most 64 items (>= 2 bytes each, <= 128-byte tokens), so counts farther
        // than that from max_items share one class.  Merging count = max-1 with count = max-2
        // would hand a mask that allows ',' after the last permitted item to the other state.
        const Node& n = nodes_[f.node];
        const int cls = (f.count < n.min_items || n.max_items - f.count <= 64) ? f.count : -1;
        k.append(reinterpret_cast<const char*>(&cls), 4);
        break;
      }
      case F_LIT:
        k.append(reinterpret_cast<const char*>(&f.aux), 4);
        break;
      case F_INT: case F_NUM:
        k.push_back((char)f.flag);
        k.append(reinterpret_cast<const char*>(&f.count), 4);
        k.append(reinterpret_cast<const char*>(&f.aux), 4);
        k.append(reinterpret_cast<const char*>(&f.val), 8);
        break;
      default: break;
    }
  }
  return k;
}

// ============================================================================ Vocab
Vocab::Vocab(const std::vector<std::string>& token_bytes, const std::vector<int>& eos_ids)
    : tokens(token_bytes), eos(eos_ids), n_((int)token_bytes.size()) {
  std::vector<int> full, spec;
  std::vector<int> plain_len(n_, -1);
  for (int i = 0; i < n_; ++i) {
    const std::string& t = tokens[i];
    if (t.empty()) continue;
    bool ok = true, special = false;
    for (unsigned char c : t) {
      if (!printable(c)) { ok = false; break; }
      if (c == '"' || c == '\\') special = true;
    }
    if (!ok) continue;
    full.push_back(i);
    max_len_ = std::max(max_len_, (int)t.size());
    if (special) spec.push_back(i);
    else plain_len[i] = (int)t.size();
  }
  build_trie(full, full_nodes, full_edges);
  build_trie(spec, spec_nodes, spec_edges);
  const int W = words();
  plain_le.assign(max_len_ + 1, std::vector<uint32_t>(W, 0u));
  for (int i = 0; i < n_; ++i) {
    if (plain_len[i] < 0) continue;
    plain_le[plain_len[i]][i >> 5] |= 1u << (i & 31);
  }
  for (int k = 1; k <= max_len_; ++k)
    for (int w = 0; w < W; ++w) plain_le[k][w] |= plain_le[k - 1][w];
}

void Vocab::build_trie(const std::vector<int>& ids, std::vector<TrieNode>& nodes, std::vector<Edge>& edges) {
  // build with child maps, then flatten into contiguous edge ranges
  struct Tmp {
    std::vector<std::pair<unsigned char, int>> ch;
    int token = -1;
  };
  std::vector<Tmp> tmp(1);
  for (int id : ids) {
    int cur = 0;
    for (unsigned char c : tokens[id]) {
      int nxt = -1;
      for (auto& e : tmp[cur].ch)
        if (e.first == c) { nxt = e.second; break; }
      if (nxt < 0) {
        nxt = (int)tmp.size();
        tmp[cur].ch.emplace_back(c, nxt);
        tmp.emplace_back();
      }
      cur = nxt;
    }
    tmp[cur].token = id;
  }
  nodes.assign(tmp.size(), TrieNode());
  edges.clear();
  for (size_t i = 0; i < tmp.size(); ++i) {
    nodes[i].token = tmp[i].token;
    nodes[i].first_child = (int)edges.size();
    nodes[i].n_children = (int)tmp[i].ch.size();
    for (auto& e : tmp[i].ch) edges.push_back(Edge{e.first, e.second});
  }
}

// ============================================================================ Compiled (mask cache)
Compiled::Compiled(std::shared_ptr<Grammar> gg, std::shared_ptr<Vocab> vv, size_t cache_cap)
    : g(std::move(gg)), v(std::move(vv)), cap_(cache_cap) {}

static inline void copy_state(State& dst, const State& src) {
  dst.depth = src.depth;
  dst.used = src.used;
  dst.done = src.done;
  std::memcpy(dst.st, src.st, sizeof(Frame) * src.depth);
}

void Compiled::dfs(const std::vector<Vocab::TrieNode>& nodes, const std::vector<Vocab::Edge>& edges, const State& s0,
                   int budget_left, std::vector<uint32_t>& out) {
  const int L = v->max_len() + 1;
  std::vector<State> st(L + 1);
  copy_state(st[0], s0);
  // iterative DFS: (trie node, depth, next edge)
  struct It { int node, depth, e; };
  std::vector<It> stack;
  stack.push_back({0, 0, 0});
  while (!stack.empty()) {
    It& it = stack.back();
    const Vocab::TrieNode& tn = nodes[it.node];
    if (it.e >= tn.n_children) {
      stack.pop_back();
      continue;
    }
    const Vocab::Edge& ed = edges[tn.first_child + it.e];
    it.e++;
    const int d = it.depth;
    State& ns = st[d + 1];
    copy_state(ns, st[d]);
    if (!g->step(ns, ed.byte)) continue;
    const Vocab::TrieNode& cn = nodes[ed.child];
    if (cn.token >= 0) {
      if ((d + 1) + g->min_completion(ns) <= budget_left) out[cn.token >> 5] |= 1u << (cn.token & 31);
    }
    if (cn.n_children > 0) stack.push_back({ed.child, d + 1, 0});
  }
}

void Compiled::compute(const State& s, int budget_left, std::vector<uint32_t>& out) {
  out.assign(v->words(), 0u);
  if (s.done) {
    for (int e : v->eos) out[e >> 5] |= 1u << (e & 31);
    return;
  }
  const Frame& top = s.st[s.depth - 1];
  if (top.kind == F_STR && !top.flag) {
    const int mc = g->min_completion(s);
    int k = std::min(top.aux - (int)top.count, budget_left - mc);
    k = std::min(k, v->max_len());
    if (k > 0) {
      const std::vector<uint32_t>& pl = v->plain_le[k];
      for (int w = 0; w < v->words(); ++w) out[w] |= pl[w];
    }
    dfs(v->spec_nodes, v->spec_edges, s, budget_left, out);
  } else {
    dfs(v->full_nodes, v->full_edges, s, budget_left, out);
  }
}

const std::vector<uint32_t>& Compiled::mask(const State& s, int budget_left) {
  const int mc = g->min_completion(s);
  const int clip = v->max_len() + 128;
  const int slack = std::min(budget_left - mc, clip);
  std::string key = g->canon(s);
  key.append(reinterpret_cast<const char*>(&slack), 4);
  auto it = cache_.find(key);
  if (it != cache_.end()) {
    ++hits;
    lru_.splice(lru_.begin(), lru_, it->second.second);
    return it->second.first;
  }
  ++misses;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<uint32_t> m;
  // compute with the clipped budget so the cached mask is valid for every budget in the class
  compute(s, slack + mc, m);
  miss_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (cache_.size() >= cap_) {
    cache_.erase(lru_.back());
    lru_.pop_back();
  }
  lru_.push_front(key);
  auto res = cache_.emplace(key, std::make_pair(std::move(m), lru_.begin()));
  return res.first->second.first;
}

// ============================================================================ Matcher
Matcher::Matcher(std::shared_ptr<Compiled> c, int budget) : c_(std::move(c)), s_(c_->g->initial()), budget_(budget) {}

bool Matcher::accept_bytes(const std::string& bytes) {
  State t;
  copy_state(t, s_);
  for (unsigned char ch : bytes)
    if (!c_->g->step(t, ch)) return false;
  if (t.used + c_->g->min_completion(t) > budget_) return false;
  copy_state(s_, t);
  return true;
}

bool Matcher::can_accept_token(int id) const {
  if (id < 0 || id >= c_->v->size()) return false;
  for (int e : c_->v->eos)
    if (e == id) return s_.done;
  const std::string& b = c_->v->tokens[id];
  if (b.empty()) return false;
  State t;
  copy_state(t, s_);
  for (unsigned char ch : b)
    if (!c_->g->step(t, ch)) return false;
  return t.used + c_->g->min_completion(t) <= budget_;
}

bool Matcher::accept_token(int id) {
  if (id < 0 || id >= c_->v->size()) return false;
  for (int e : c_->v->eos)
    if (e == id) return s_.done;
  const std::string& b = c_->v->tokens[id];
  if (b.empty()) return false;
  return accept_bytes(b);
}

void Matcher::fill_mask(uint32_t* out) const {
  const std::vector<uint32_t>& m = c_->mask(s_, budget_ - s_.used);
  std::memcpy(out, m.data(), m.size() * sizeof(uint32_t));
}

std::string Matcher::forced_prefix(int max_len) const {
  std::string out;
  State cur;
  copy_state(cur, s_);
  State t;
  while ((int)out.size() < max_len && !cur.done) {
    int n_ok = 0;
    unsigned char only = 0;
    for (int c = 0x20; c <= 0x7e && n_ok < 2; ++c) {
      copy_state(t, cur);
      if (c_->g->step(t, (unsigned char)c) && t.used + c_->g->min_completion(t) <= budget_) {
        ++n_ok;
        only = (unsigned char)c;
      }
    }
    if (n_ok != 1) break;
    c_->g->step(cur, only);
    out.push_back((char)only);
  }
  return out;
}

}  // namespace vwa
