// JSON-schema constrained decoding engine (CPU side of K13).
//
// Replaces the reference's `response_format: {type: "json_object"}` + zod validation + one
// repair call (apps/brain/src/llm.ts:25, apps/brain/src/server.ts:107-136): instead of asking a
// hosted model for JSON and repairing it afterwards, every decode step is masked so that only
// tokens keeping the output a valid prefix of a ParseResponse are sampleable.  A random-init
// model therefore always produces schema-valid intents.
//
// Pieces:
//  * Grammar  : schema IR (objects with ordered/optional keys, free-form records, arrays with
//               item bounds, bounded strings, enums, constants, ranged ints/decimals, bool,
//               null, alternatives), parsed from a compact JSON description.
//  * State    : character-level pushdown matcher; fixed-capacity POD stack so a state copy is a
//               small memcpy (the mask DFS copies one per trie node).
//  * Vocab    : raw bytes of every token + a byte trie; "plain" tokens (printable ASCII without
//               '"' or '\\') are indexed by length so the dominant free-string state is served
//               by a precomputed bitset; only "special" tokens are walked through the matcher.
//  * Masker   : mask = union over tokens that keep the state valid AND leave enough character
//               budget to close the JSON (min_completion), cached per canonical state.
//  * forced_prefix: jump-forward -- the unique continuation bytes when only one is legal.
#pragma once
#include <cstdint>
#include <cstring>
#include <list>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

namespace vwa {

enum NodeKind : uint8_t { N_OBJ, N_REC, N_ARR, N_STR, N_ENUM, N_CONST, N_INT, N_NUM, N_BOOL, N_NULL, N_ALT };

struct Prop {
  std::string key;  // raw key text (without quotes)
  int node;
  bool required;
};

struct Node {
  NodeKind kind;
  // OBJ
  std::vector<Prop> props;
  std::vector<int> rest_after;  // rest_after[j]: min chars for required props after j (incl commas)
  // REC / ARR
  int item = -1;  // REC value node / ARR item node
  int min_items = 0, max_items = 0;
  int key_max = 0;  // REC key max length
  // STR
  int max_len = 0;
  // ENUM / CONST
  std::vector<std::string> values;  // ENUM values (raw, no quotes) / CONST text
  // INT / NUM
  double lo = 0, hi = 0;
  int frac = 0;
  // ALT
  std::vector<int> opts;
  // derived
  int min_len = 0;
  int lit = -1;                  // CONST: literal id
  uint8_t first[256 / 8] = {0};  // first-char set
};

enum FrameKind : uint8_t { F_VALUE, F_OBJ, F_REC, F_ARR, F_STR, F_ENUM, F_LIT, F_INT, F_NUM };

constexpr int kBuf = 30;
constexpr int kMaxDepth = 12;

struct Frame {
  uint8_t kind;
  uint8_t phase;
  uint8_t blen;     // used bytes of buf
  uint8_t flag;     // escape pending / negative / in-fraction ...
  int16_t node;
  int16_t idx;      // OBJ: current/next prop index; LIT: position
  int32_t count;    // REC/ARR items; STR length; INT/NUM digits
  int32_t aux;      // NUM fraction digits
  double val;       // INT/NUM magnitude so far
  char buf[kBuf];   // OBJ key prefix / ENUM prefix / LIT literal id
};

struct State {
  int depth = 0;
  int used = 0;       // bytes emitted so far
  bool done = false;  // top-level value complete
  Frame st[kMaxDepth];
};

class Grammar {
 public:
  explicit Grammar(const std::string& ir_json);
  int root() const { return root_; }
  const Node& node(int i) const { return nodes_[i]; }
  int n_nodes() const { return (int)nodes_.size(); }
  // literal table for F_LIT frames
  int lit_id(const std::string& s);
  const std::string& lit(int id) const { return lits_[id]; }

  State initial() const;
  bool step(State& s, unsigned char c) const;
  int min_completion(const State& s) const;
  bool is_accept(const State& s) const { return s.done; }
  std::string canon(const State& s) const;

 private:
  void finalize();
  int node_min_len(int i, std::vector<int>& visiting);
  void compute_first(int i, std::vector<int>& visiting);
  bool push_value(State& s, int node, unsigned char c) const;
  bool feed(State& s, unsigned char c) const;
  void pop(State& s) const;
  int frame_remaining(const Frame& f) const;

  std::vector<Node> nodes_;
  std::vector<std::string> lits_;
  int root_ = 0;
  int lit_true_ = -1, lit_false_ = -1, lit_null_ = -1;
};

class Vocab {
 public:
  Vocab(const std::vector<std::string>& token_bytes, const std::vector<int>& eos_ids);
  int size() const { return n_; }
  int words() const { return (n_ + 31) / 32; }
  int max_len() const { return max_len_; }

  struct TrieNode {
    int first_child = -1;  // index into edges
    int n_children = 0;
    int token = -1;        // token id ending here (-1 none)
  };
  struct Edge {
    unsigned char byte;
    int child;
  };
  std::vector<std::string> tokens;
  std::vector<int> eos;
  // full trie (all normal tokens) and special trie (printable tokens containing '"' or '\\')
  std::vector<TrieNode> full_nodes, spec_nodes;
  std::vector<Edge> full_edges, spec_edges;
  // plain_le[k]: bitset of plain tokens (printable, no quote/backslash) of byte length <= k
  std::vector<std::vector<uint32_t>> plain_le;

 private:
  void build_trie(const std::vector<int>& ids, std::vector<TrieNode>& nodes, std::vector<Edge>& edges);
  int n_ = 0;
  int max_len_ = 0;
};

class Matcher;

class Compiled {
 public:
  Compiled(std::shared_ptr<Grammar> g, std::shared_ptr<Vocab> v, size_t cache_cap = 4096);
  std::shared_ptr<Grammar> g;
  std::shared_ptr<Vocab> v;
  // mask for state s with `budget_left` bytes remaining (total budget - used)
  const std::vector<uint32_t>& mask(const State& s, int budget_left);
  size_t hits = 0, misses = 0;
  double miss_ms = 0.0;

 private:
  void compute(const State& s, int budget_left, std::vector<uint32_t>& out);
  void dfs(const std::vector<Vocab::TrieNode>& nodes, const std::vector<Vocab::Edge>& edges, const State& s0,
           int budget_left, std::vector<uint32_t>& out);
  size_t cap_;
  std::list<std::string> lru_;
  std::unordered_map<std::string, std::pair<std::vector<uint32_t>, std::list<std::string>::iterator>> cache_;
};

class Matcher {
 public:
  Matcher(std::shared_ptr<Compiled> c, int budget);
  bool accept_bytes(const std::string& bytes);
  bool accept_token(int id);
  bool can_accept_token(int id) const;
  void fill_mask(uint32_t* out) const;
  std::string forced_prefix(int max_len = 256) const;
  bool is_accept() const { return c_->g->is_accept(s_); }
  int used() const { return s_.used; }
  int min_completion() const { return c_->g->min_completion(s_); }
  int budget() const { return budget_; }
  std::string canon() const { return c_->g->canon(s_); }
  Matcher clone() const { return *this; }
  std::shared_ptr<Compiled> compiled() const { return c_; }

 private:
  std::shared_ptr<Compiled> c_;
  State s_;
  int budget_;
};

}  // namespace vwa
