// ingest.cpp — non-executing parser for pickled Plato state_dict payloads and
// a multi-threaded gather into flat (pinned) arenas.  C ABI: include/plato_ingest.h.
//
// The interpreter understands the pickle opcodes that pickle.dumps (protocols
// 2-5) emits for a dict / OrderedDict of CPU tensors and the legacy
// torch.save records inside torch.storage._load_from_bytes.  It builds no
// Python objects and calls nothing: REDUCE is only accepted for the three
// whitelisted callables, everything else is rejected.  All reads are bounds
// checked against [buf, buf + len).
#include <dlfcn.h>
#include <unistd.h>

#include <cerrno>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "plato_ingest.h"

namespace {

thread_local std::string g_err;

struct Error {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }

// ---------------------------------------------------------------- values
enum class K { None, Bool, Int, Float, Str, Bytes, Global, Tuple, List, Dict, Mark, Storage, Tensor };

struct Val;
// Values are owned by the parse's Ctx::pool and referenced by raw pointer:
// a hostile pickle can nest containers arbitrarily deep or build reference
// cycles (memo GET + APPEND), and a pool is freed iteratively either way
// (shared_ptr chains would recurse on destruction and leak on cycles).
using P = Val*;

struct Val {
  K k = K::None;
  int64_t i = 0;           // Int / Bool / Storage id / Tensor index
  double f = 0;            // Float
  uint64_t off = 0, len = 0;  // Str / Bytes: view into the buffer
  std::string mod, name;   // Global
  std::vector<P> items;    // Tuple / List
  std::vector<std::pair<P, P>> dict;  // Dict (insertion order)
};


struct Storage {
  int32_t dtype = -1;
  int32_t elem = 0;
  uint64_t numel = 0;
  uint64_t data_offset = 0;
  bool has_data = false;
  std::string key;
};

struct Ctx {
  const uint8_t* buf;
  size_t len;
  std::vector<Storage> storages;
  std::vector<plato_ingest_tensor> tensors;
  std::vector<std::unique_ptr<Val>> pool;  // every Val of this parse
  int record_depth = 0;                     // nested _load_from_bytes records

  std::string str(const Val& v) const { return std::string(reinterpret_cast<const char*>(buf + v.off), v.len); }
};

struct Reader {
  const Ctx& c;
  size_t pos, end;
  void need(size_t n) const {
    if (n > end - pos) fail(PLATO_INGEST_EFORMAT, "truncated pickle");
  }
  uint8_t u8() {
    need(1);
    return c.buf[pos++];
  }
  uint64_t le(int n) {
    need(size_t(n));
    uint64_t v = 0;
    for (int b = 0; b < n; ++b) v |= uint64_t(c.buf[pos + b]) << (8 * b);
    pos += size_t(n);
    return v;
  }
  std::string line() {
    size_t q = pos;
    while (q < end && c.buf[q] != '\n') ++q;
    if (q >= end) fail(PLATO_INGEST_EFORMAT, "unterminated GLOBAL line");
    std::string s(reinterpret_cast<const char*>(c.buf + pos), q - pos);
    pos = q + 1;
    return s;
  }
};

P mk(Ctx& c, K k) {
  c.pool.push_back(std::make_unique<Val>());
  P p = c.pool.back().get();
  p->k = k;
  return p;
}

int dtype_of_storage(const std::string& mod, const std::string& name, int32_t* elem) {
  if (mod != "torch") return -1;
  static const struct {
    const char* n;
    int dt, es;
  } table[] = {{"FloatStorage", PLATO_DT_F32, 4}, {"LongStorage", PLATO_DT_I64, 8},
               {"DoubleStorage", PLATO_DT_F64, 8}, {"HalfStorage", PLATO_DT_F16, 2},
               {"BFloat16Storage", PLATO_DT_BF16, 2}, {"IntStorage", PLATO_DT_I32, 4},
               {"ShortStorage", PLATO_DT_I16, 2}, {"CharStorage", PLATO_DT_I8, 1},
               {"ByteStorage", PLATO_DT_U8, 1}, {"BoolStorage", PLATO_DT_BOOL, 1}};
  for (const auto& t : table) {
    if (name == t.n) {
      *elem = t.es;
      return t.dt;
    }
  }
  return -1;
}

int64_t as_int(const P& v, const char* what) {
  if (!v || (v->k != K::Int && v->k != K::Bool)) fail(PLATO_INGEST_EUNSUPPORTED, std::string(what) + ": expected int");
  return v->i;
}

// ------------------------------------------------------------ interpreter
struct Persistent {
  // legacy torch.save persistent ids -> storage index
  std::unordered_map<std::string, int> by_key;
};

P parse_legacy_record(Ctx& c, uint64_t off, uint64_t len);
bool tensor_in_storage(const plato_ingest_tensor& t);

// Runs one pickle from r.pos to its STOP; returns the top of the stack.
P run(Ctx& c, Reader& r, Persistent* pers) {
  std::vector<P> st;
  std::vector<size_t> marks;
  std::vector<P> memo;
  auto pop = [&]() -> P {
    if (st.empty()) fail(PLATO_INGEST_EFORMAT, "stack underflow");
    P v = st.back();
    st.pop_back();
    return v;
  };
  auto pop_mark = [&]() -> std::vector<P> {
    if (marks.empty()) fail(PLATO_INGEST_EFORMAT, "no MARK");
    size_t m = marks.back();
    marks.pop_back();
    if (m > st.size()) fail(PLATO_INGEST_EFORMAT, "bad MARK");
    std::vector<P> items(st.begin() + long(m), st.end());
    st.resize(m);
    return items;
  };
  auto memo_put = [&](size_t idx) {
    if (st.empty()) fail(PLATO_INGEST_EFORMAT, "PUT on empty stack");
    if (idx > (size_t(1) << 24)) fail(PLATO_INGEST_EUNSUPPORTED, "memo index too large");
    if (memo.size() <= idx) memo.resize(idx + 1);
    memo[idx] = st.back();
  };
  auto memo_get = [&](size_t idx) {
    if (idx >= memo.size() || !memo[idx]) fail(PLATO_INGEST_EFORMAT, "GET of unset memo");
    st.push_back(memo[idx]);
  };
  auto push_view = [&](K k, uint64_t n) {
    r.need(size_t(n));
    P v = mk(c, k);
    v->off = r.pos;
    v->len = n;
    r.pos += size_t(n);
    st.push_back(v);
  };
  auto set_items = [&](const P& d, const std::vector<P>& kv) {
    if (!d || d->k != K::Dict) fail(PLATO_INGEST_EUNSUPPORTED, "SETITEMS on a non-dict");
    if (kv.size() % 2) fail(PLATO_INGEST_EFORMAT, "odd SETITEMS");
    for (size_t j = 0; j < kv.size(); j += 2) d->dict.emplace_back(kv[j], kv[j + 1]);
  };

  for (;;) {
    const uint8_t op = r.u8();
    switch (op) {
      case 0x80: r.u8(); break;                       // PROTO
      case 0x95: r.le(8); break;                      // FRAME (transparent)
      case '.': return st.empty() ? mk(c, K::None) : st.back();  // STOP
      case '(': marks.push_back(st.size()); break;    // MARK
      case '}': st.push_back(mk(c, K::Dict)); break;     // EMPTY_DICT
      case ']': st.push_back(mk(c, K::List)); break;     // EMPTY_LIST
      case ')': st.push_back(mk(c, K::Tuple)); break;    // EMPTY_TUPLE
      case 't': {                                     // TUPLE
        P t = mk(c, K::Tuple);
        t->items = pop_mark();
        st.push_back(t);
        break;
      }
      case 0x85: case 0x86: case 0x87: {              // TUPLE1..3
        const int n = op - 0x84;
        if (st.size() < size_t(n)) fail(PLATO_INGEST_EFORMAT, "stack underflow");
        P t = mk(c, K::Tuple);
        t->items.assign(st.end() - n, st.end());
        st.resize(st.size() - size_t(n));
        st.push_back(t);
        break;
      }
      case 'a': {                                     // APPEND
        P v = pop();
        if (st.empty() || st.back()->k != K::List) fail(PLATO_INGEST_EUNSUPPORTED, "APPEND to non-list");
        st.back()->items.push_back(v);
        break;
      }
      case 'e': {                                     // APPENDS
        auto items = pop_mark();
        if (st.empty() || st.back()->k != K::List) fail(PLATO_INGEST_EUNSUPPORTED, "APPENDS to non-list");
        for (auto& v : items) st.back()->items.push_back(v);
        break;
      }
      case 's': {                                     // SETITEM
        P v = pop();
        P k = pop();
        if (st.empty()) fail(PLATO_INGEST_EFORMAT, "stack underflow");
        set_items(st.back(), {k, v});
        break;
      }
      case 'u': {                                     // SETITEMS
        auto kv = pop_mark();
        if (st.empty()) fail(PLATO_INGEST_EFORMAT, "stack underflow");
        set_items(st.back(), kv);
        break;
      }
      case 'J': { P v = mk(c, K::Int); v->i = int32_t(uint32_t(r.le(4))); st.push_back(v); break; }
      case 'K': { P v = mk(c, K::Int); v->i = r.u8(); st.push_back(v); break; }
      case 'M': { P v = mk(c, K::Int); v->i = int64_t(r.le(2)); st.push_back(v); break; }
      case 0x8a: case 0x8b: {                         // LONG1 / LONG4
        const uint64_t n = op == 0x8a ? r.u8() : r.le(4);
        r.need(size_t(n));
        P v = mk(c, K::Int);
        v->off = r.pos;
        if (n > 8) {
          // only the legacy magic number is this long: keep its low bits
          uint64_t lo = 0;
          for (int b = 0; b < 8; ++b) lo |= uint64_t(c.buf[r.pos + size_t(b)]) << (8 * b);
          v->i = int64_t(lo);
          v->len = n;
        } else if (n > 0) {
          uint64_t x = 0;
          for (uint64_t b = 0; b < n; ++b) x |= uint64_t(c.buf[r.pos + size_t(b)]) << (8 * b);
          if (n < 8 && (c.buf[r.pos + size_t(n) - 1] & 0x80)) x |= ~uint64_t(0) << (8 * n);  // sign extend
          v->i = int64_t(x);
        }
        r.pos += size_t(n);
        st.push_back(v);
        break;
      }
      case 'N': st.push_back(mk(c, K::None)); break;
      case 0x88: { P v = mk(c, K::Bool); v->i = 1; st.push_back(v); break; }
      case 0x89: { P v = mk(c, K::Bool); v->i = 0; st.push_back(v); break; }
      case 'G': {                                     // BINFLOAT (big endian)
        r.need(8);
        uint64_t x = 0;
        for (int b = 0; b < 8; ++b) x = (x << 8) | c.buf[r.pos + size_t(b)];
        r.pos += 8;
        P v = mk(c, K::Float);
        std::memcpy(&v->f, &x, 8);
        st.push_back(v);
        break;
      }
      case 0x8c: push_view(K::Str, r.u8()); break;    // SHORT_BINUNICODE
      case 'X': push_view(K::Str, r.le(4)); break;    // BINUNICODE
      case 0x8d: push_view(K::Str, r.le(8)); break;   // BINUNICODE8
      case 'U': push_view(K::Str, r.u8()); break;     // SHORT_BINSTRING
      case 'T': push_view(K::Str, r.le(4)); break;    // BINSTRING
      case 'C': push_view(K::Bytes, r.u8()); break;   // SHORT_BINBYTES
      case 'B': push_view(K::Bytes, r.le(4)); break;  // BINBYTES
      case 0x8e: push_view(K::Bytes, r.le(8)); break; // BINBYTES8
      case 0x96: push_view(K::Bytes, r.le(8)); break; // BYTEARRAY8
      case 0x94: memo_put(memo.size()); break;        // MEMOIZE
      case 'q': memo_put(r.u8()); break;              // BINPUT
      case 'r': memo_put(size_t(r.le(4))); break;     // LONG_BINPUT
      case 'h': memo_get(r.u8()); break;              // BINGET
      case 'j': memo_get(size_t(r.le(4))); break;     // LONG_BINGET
      case 'c': {                                     // GLOBAL
        P g = mk(c, K::Global);
        g->mod = r.line();
        g->name = r.line();
        st.push_back(g);
        break;
      }
      case 0x93: {                                    // STACK_GLOBAL
        P name = pop();
        P mod = pop();
        if (mod->k != K::Str || name->k != K::Str) fail(PLATO_INGEST_EFORMAT, "STACK_GLOBAL needs strings");
        P g = mk(c, K::Global);
        g->mod = c.str(*mod);
        g->name = c.str(*name);
        st.push_back(g);
        break;
      }
      case 'Q': {                                     // BINPERSID (legacy torch.save)
        P pid = pop();
        if (!pers) fail(PLATO_INGEST_EUNSUPPORTED, "persistent id outside a torch record");
        if (pid->k != K::Tuple || pid->items.size() < 5 || pid->items[0]->k != K::Str ||
            c.str(*pid->items[0]) != "storage")
          fail(PLATO_INGEST_EUNSUPPORTED, "unexpected persistent id");
        const P& type = pid->items[1];
        const P& key = pid->items[2];
        if (type->k != K::Global || key->k != K::Str) fail(PLATO_INGEST_EUNSUPPORTED, "bad storage id");
        Storage s;
        s.dtype = dtype_of_storage(type->mod, type->name, &s.elem);
        if (s.dtype < 0) fail(PLATO_INGEST_EUNSUPPORTED, "storage type " + type->mod + "." + type->name);
        const int64_t numel = as_int(pid->items[4], "storage numel");
        if (numel < 0) fail(PLATO_INGEST_EFORMAT, "negative storage size");
        s.numel = uint64_t(numel);
        s.key = c.str(*key);
        auto it = pers->by_key.find(s.key);
        int idx;
        if (it == pers->by_key.end()) {
          idx = int(c.storages.size());
          c.storages.push_back(s);
          pers->by_key.emplace(s.key, idx);
        } else {
          idx = it->second;
        }
        P v = mk(c, K::Storage);
        v->i = idx;
        st.push_back(v);
        break;
      }
      case 'R': {                                     // REDUCE (whitelist)
        P args = pop();
        P fn = pop();
        if (fn->k != K::Global || args->k != K::Tuple) fail(PLATO_INGEST_EUNSUPPORTED, "REDUCE of a non-global");
        if ((fn->mod == "collections" && fn->name == "OrderedDict") && args->items.empty()) {
          st.push_back(mk(c, K::Dict));
        } else if (fn->mod == "torch.storage" && fn->name == "_load_from_bytes") {
          if (args->items.size() != 1 || args->items[0]->k != K::Bytes)
            fail(PLATO_INGEST_EFORMAT, "_load_from_bytes(bytes) expected");
          st.push_back(parse_legacy_record(c, args->items[0]->off, args->items[0]->len));
        } else if (fn->mod == "torch._utils" && fn->name == "_rebuild_tensor_v2") {
          const auto& a = args->items;
          if (a.size() < 5 || a[0]->k != K::Storage || a[2]->k != K::Tuple || a[3]->k != K::Tuple)
            fail(PLATO_INGEST_EFORMAT, "_rebuild_tensor_v2 arguments");
          const Storage& s = c.storages[size_t(a[0]->i)];
          plato_ingest_tensor t;
          std::memset(&t, 0, sizeof(t));
          t.dtype = s.dtype;
          t.element_size = s.elem;
          t.storage_id = int32_t(a[0]->i);
          t.storage_numel = s.numel;
          const int64_t so = as_int(a[1], "storage offset");
          if (so < 0) fail(PLATO_INGEST_EFORMAT, "negative storage offset");
          t.storage_offset = uint64_t(so);
          const size_t nd = a[2]->items.size();
          if (nd > PLATO_INGEST_MAX_DIMS || a[3]->items.size() != nd)
            fail(PLATO_INGEST_EUNSUPPORTED, "tensor rank > 8 or size/stride mismatch");
          t.ndim = int32_t(nd);
          uint64_t numel = 1;
          bool contig = true;
          int64_t expect = 1;
          for (size_t d = 0; d < nd; ++d) {
            const int64_t sz = as_int(a[2]->items[d], "size");
            const int64_t sd = as_int(a[3]->items[d], "stride");
            if (sz < 0 || sd < 0) fail(PLATO_INGEST_EFORMAT, "negative size/stride");
            t.shape[d] = sz;
            t.stride[d] = sd;
            if (sz != 0 && numel > (uint64_t(1) << 48) / uint64_t(sz)) fail(PLATO_INGEST_EFORMAT, "tensor too large");
            numel *= uint64_t(sz);
          }
          for (size_t d = nd; d-- > 0;) {
            if (t.shape[d] != 1 && t.stride[d] != expect) contig = false;
            expect *= t.shape[d];
          }
          t.numel = numel;
          t.contiguous = contig ? 1 : 0;
          if (!tensor_in_storage(t)) fail(PLATO_INGEST_EFORMAT, "tensor outside its storage");
          P v = mk(c, K::Tensor);
          v->i = int64_t(c.tensors.size());
          c.tensors.push_back(t);
          st.push_back(v);
        } else {
          fail(PLATO_INGEST_EUNSUPPORTED, "REDUCE of " + fn->mod + "." + fn->name);
        }
        break;
      }
      default: {
        char hex[8];
        std::snprintf(hex, sizeof(hex), "0x%02x", op);
        fail(PLATO_INGEST_EUNSUPPORTED, std::string("pickle opcode ") + hex);
      }
    }
  }
}

// torch.save(storage, _use_new_zipfile_serialization=False) record.
P parse_legacy_record(Ctx& c, uint64_t off, uint64_t len) {
  // A state_dict pickle holds records one level deep; a record whose storage
  // pickle calls _load_from_bytes again is never produced by torch.
  struct Depth {
    Ctx& c;
    explicit Depth(Ctx& cc) : c(cc) {
      if (++c.record_depth > 2) fail(PLATO_INGEST_EUNSUPPORTED, "nested torch.save records");
    }
    ~Depth() { --c.record_depth; }
  } depth(c);
  Reader r{c, size_t(off), size_t(off + len)};
  Persistent pers;
  P magic = run(c, r, nullptr);
  static const uint8_t kMagic[10] = {0x6c, 0xfc, 0x9c, 0x46, 0xf9, 0x20, 0x6a, 0xa8, 0x50, 0x19};
  if (magic->k != K::Int || magic->len != 10 || std::memcmp(c.buf + magic->off, kMagic, 10) != 0)
    fail(PLATO_INGEST_EUNSUPPORTED, "not a legacy torch.save record");
  P proto = run(c, r, nullptr);
  if (proto->k != K::Int || proto->i != 1001) fail(PLATO_INGEST_EUNSUPPORTED, "torch.save protocol != 1001");
  P info = run(c, r, nullptr);  // sys info: little_endian must not be False
  if (info->k == K::Dict) {
    for (auto& kv : info->dict) {
      if (kv.first->k == K::Str && c.str(*kv.first) == "little_endian" && kv.second->k == K::Bool && !kv.second->i)
        fail(PLATO_INGEST_EUNSUPPORTED, "big-endian record");
    }
  }
  P obj = run(c, r, &pers);
  P keys = run(c, r, nullptr);
  if (keys->k != K::List) fail(PLATO_INGEST_EFORMAT, "storage key list expected");
  for (auto& k : keys->items) {
    if (k->k != K::Str) fail(PLATO_INGEST_EFORMAT, "storage key not a string");
    auto it = pers.by_key.find(c.str(*k));
    if (it == pers.by_key.end()) fail(PLATO_INGEST_EFORMAT, "unknown storage key");
    Storage& s = c.storages[size_t(it->second)];
    const uint64_t numel = r.le(8);
    if (numel != s.numel) fail(PLATO_INGEST_EFORMAT, "storage size mismatch");
    const uint64_t bytes = numel * uint64_t(s.elem);
    if (s.elem && numel > (~uint64_t(0)) / uint64_t(s.elem)) fail(PLATO_INGEST_EFORMAT, "storage too large");
    r.need(size_t(bytes));
    s.data_offset = r.pos;
    s.has_data = true;
    r.pos += size_t(bytes);
  }
  if (obj->k != K::Storage || !c.storages[size_t(obj->i)].has_data)
    fail(PLATO_INGEST_EFORMAT, "record holds no storage data");
  return obj;
}

// --------------------------------------------------------------- gather
struct Piece {
  const uint8_t* src;
  uint8_t* dst;
  size_t bytes;
};

// Persistent copy workers: creating threads in every gather call cost more
// than the copies (~20 us per thread, two gathers per payload).
class Pool {
 public:
  static Pool& get() {
    static Pool* p = new Pool();  // never destroyed: no teardown ordering at exit
    return *p;
  }

  // Runs fn(0 .. n_tasks-1) on up to `width` threads, the caller included.
  void run(size_t n_tasks, int width, const std::function<void(size_t)>& fn) {
    std::lock_guard<std::mutex> call(call_mu_);  // one parallel gather at a time
    const int helpers = std::max(0, std::min(width, kMax) - 1);
    std::atomic<size_t> next{0};
    std::function<void()> body = [&]() {
      for (size_t k = next.fetch_add(1); k < n_tasks; k = next.fetch_add(1)) fn(k);
    };
    {
      std::lock_guard<std::mutex> lk(mu_);
      while (int(spawned_) < helpers) {
        const int id = spawned_++;
        std::thread([this, id] { loop(id); }).detach();
      }
      job_ = &body;
      participants_ = helpers;
      remaining_ = helpers;
      ++gen_;
    }
    cv_.notify_all();
    body();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return remaining_ == 0; });
    job_ = nullptr;
  }

 private:
  static constexpr int kMax = 32;

  void loop(int id) {
    uint64_t seen = 0;
    for (;;) {
      std::function<void()>* job = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (id >= participants_) continue;
        job = job_;
      }
      (*job)();
      {
        std::lock_guard<std::mutex> lk(mu_);
        --remaining_;
      }
      done_cv_.notify_all();
    }
  }

  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::function<void()>* job_ = nullptr;
  int spawned_ = 0;
  int participants_ = 0;
  int remaining_ = 0;
  uint64_t gen_ = 0;
};

// True when every element of t lies inside its storage: storage_offset +
// sum((shape[d]-1) * stride[d]) < storage_numel, with no step of the sum
// wrapping (a hostile record may carry strides up to 2^63-1), and numel equal
// to the product of the shape.  Checked by the parser and again by the gather
// (its descriptors come through the C ABI).
bool tensor_in_storage(const plato_ingest_tensor& t) {
  if (t.ndim < 0 || t.ndim > PLATO_INGEST_MAX_DIMS) return false;
  uint64_t numel = 1, span = 0;
  for (int d = 0; d < t.ndim; ++d) {
    if (t.shape[d] < 0 || t.stride[d] < 0) return false;
    if (__builtin_mul_overflow(numel, uint64_t(t.shape[d]), &numel)) return false;
  }
  if (numel != t.numel) return false;
  if (numel == 0) return true;  // an empty tensor reads nothing, whatever its strides
  for (int d = 0; d < t.ndim; ++d) {
    if (t.shape[d] > 1) {
      uint64_t ext = 0;
      if (uint64_t(t.stride[d]) >= t.storage_numel) return false;
      if (__builtin_mul_overflow(uint64_t(t.shape[d] - 1), uint64_t(t.stride[d]), &ext) ||
          __builtin_add_overflow(span, ext, &span))
        return false;
    }
  }
  uint64_t last = 0;
  return !__builtin_add_overflow(t.storage_offset, span, &last) && last < t.storage_numel;
}

void copy_strided(const uint8_t* base, const plato_ingest_tensor& t, uint8_t* dst) {
  const size_t es = size_t(t.element_size);
  int64_t idx[PLATO_INGEST_MAX_DIMS] = {0};
  for (uint64_t n = 0; n < t.numel; ++n) {
    uint64_t e = t.storage_offset;
    for (int d = 0; d < t.ndim; ++d) e += uint64_t(idx[d]) * uint64_t(t.stride[d]);
    std::memcpy(dst + n * es, base + e * es, es);
    for (int d = t.ndim - 1; d >= 0; --d) {
      if (++idx[d] < t.shape[d]) break;
      idx[d] = 0;
    }
  }
}

// ----------------------------------------------------------------- zstd
// Plato's model_compress / model_decompress processors wrap the pickled
// payload in zstd frames (python-zstd's compress: a standard frame with the
// content size in its header).  The codec is the system libzstd.so.1, bound
// at first use with dlopen, so the library has no link-time dependency on it
// (parse and gather work without it).  Only stable public entry points of the
// zstd ABI are used.
struct ZstdInBuf {
  const void* src;
  size_t size;
  size_t pos;
};
struct ZstdOutBuf {
  void* dst;
  size_t size;
  size_t pos;
};

struct Zstd {
  size_t (*decompress)(void*, size_t, const void*, size_t) = nullptr;
  size_t (*compress)(void*, size_t, const void*, size_t, int) = nullptr;
  size_t (*bound)(size_t) = nullptr;
  unsigned long long (*find_size)(const void*, size_t) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
  const char* (*error_name)(size_t) = nullptr;
  void* (*create_dctx)() = nullptr;
  size_t (*free_dctx)(void*) = nullptr;
  size_t (*decompress_stream)(void*, ZstdOutBuf*, ZstdInBuf*) = nullptr;
  std::string load_error;

  static const Zstd& get() {
    static Zstd* z = load();  // never destroyed: no teardown ordering at exit
    return *z;
  }

  bool ok() const { return decompress != nullptr; }

 private:
  static Zstd* load() {
    Zstd* z = new Zstd();
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      z->load_error = std::string("libzstd.so.1 not loadable: ") + (e ? e : "?");
      return z;
    }
    bool all = true;
    auto bind = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) all = false;
    };
    decltype(z->decompress) d = nullptr;
    bind(d, "ZSTD_decompress");
    bind(z->compress, "ZSTD_compress");
    bind(z->bound, "ZSTD_compressBound");
    bind(z->find_size, "ZSTD_findDecompressedSize");
    bind(z->is_error, "ZSTD_isError");
    bind(z->error_name, "ZSTD_getErrorName");
    bind(z->create_dctx, "ZSTD_createDCtx");
    bind(z->free_dctx, "ZSTD_freeDCtx");
    bind(z->decompress_stream, "ZSTD_decompressStream");
    if (!all) {
      z->load_error = "libzstd.so.1 lacks an expected ZSTD_* entry point";
      return z;
    }
    z->decompress = d;  // set last: ok() means every entry point is bound
    return z;
  }
};

constexpr unsigned long long kZstdUnknown = ~0ull;        // ZSTD_CONTENTSIZE_UNKNOWN
constexpr unsigned long long kZstdSizeError = ~0ull - 1;  // ZSTD_CONTENTSIZE_ERROR

const Zstd* zstd_or_fail() {
  const Zstd& z = Zstd::get();
  if (!z.ok()) {
    g_err = z.load_error;
    return nullptr;
  }
  return &z;
}

// Frames without a content size (streaming compressors): decode until the
// input is consumed; the destination must be large enough.
int64_t zstd_stream(const Zstd& z, const uint8_t* src, size_t len, uint8_t* dst, size_t cap) {
  void* dctx = z.create_dctx();
  if (!dctx) {
    g_err = "ZSTD_createDCtx failed";
    return PLATO_INGEST_EFORMAT;
  }
  ZstdInBuf in{src, len, 0};
  ZstdOutBuf out{dst, cap, 0};
  size_t r = 1;
  int64_t rc = 0;
  for (;;) {
    const size_t in0 = in.pos, out0 = out.pos;
    r = z.decompress_stream(dctx, &out, &in);
    if (z.is_error(r)) {
      g_err = std::string("zstd: ") + z.error_name(r);
      rc = PLATO_INGEST_EFORMAT;
      break;
    }
    if (in.pos == in.size && r == 0) break;  // every frame complete
    if (out.pos == out.size && (in.pos < in.size || r != 0)) {
      g_err = "destination too small for the decompressed payload";
      rc = PLATO_INGEST_ECAPACITY;
      break;
    }
    if (in.pos == in0 && out.pos == out0) {
      g_err = "truncated zstd frame";
      rc = PLATO_INGEST_EFORMAT;
      break;
    }
  }
  z.free_dctx(dctx);
  if (rc < 0) return rc;
  g_err.clear();
  return int64_t(out.pos);
}

}  // namespace

extern "C" {

const char* plato_ingest_last_error(void) { return g_err.c_str(); }

int plato_ingest_zstd_available(void) { return zstd_or_fail() ? 1 : 0; }

int64_t plato_ingest_zstd_content_size(const uint8_t* src, size_t len) {
  const Zstd* z = zstd_or_fail();
  if (!z) return PLATO_INGEST_ENOCODEC;
  if (!src) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  if (len == 0) {
    g_err = "empty input: no zstd frame";
    return PLATO_INGEST_EFORMAT;
  }
  const unsigned long long n = z->find_size(src, len);
  if (n == kZstdUnknown) {
    g_err = "zstd frame without a content size";
    return PLATO_INGEST_EUNKNOWNSIZE;
  }
  if (n == kZstdSizeError || n > (unsigned long long)INT64_MAX) {
    g_err = "not a complete sequence of zstd frames";
    return PLATO_INGEST_EFORMAT;
  }
  g_err.clear();
  return int64_t(n);
}

int64_t plato_ingest_zstd_decompress(const uint8_t* src, size_t len, uint8_t* dst, size_t cap) {
  const Zstd* z = zstd_or_fail();
  if (!z) return PLATO_INGEST_ENOCODEC;
  if (!src || (cap && !dst)) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  if (len == 0) {
    g_err = "empty input: no zstd frame";
    return PLATO_INGEST_EFORMAT;
  }
  const unsigned long long n = z->find_size(src, len);
  if (n == kZstdUnknown) return zstd_stream(*z, src, len, dst, cap);
  if (n == kZstdSizeError) {
    g_err = "not a complete sequence of zstd frames";
    return PLATO_INGEST_EFORMAT;
  }
  if (n > cap) {
    g_err = "destination smaller than the frames' content size";
    return PLATO_INGEST_ECAPACITY;
  }
  const size_t r = z->decompress(dst, cap, src, len);
  if (z->is_error(r)) {
    g_err = std::string("zstd: ") + z->error_name(r);
    return PLATO_INGEST_EFORMAT;
  }
  g_err.clear();
  return int64_t(r);
}

int plato_ingest_join(const uint8_t* const* chunks, const size_t* lens, int n, uint8_t* dst, size_t dst_len,
                      int threads) {
  if (n < 0 || (n > 0 && (!chunks || !lens)) || (!dst && dst_len)) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  std::vector<Piece> pieces;
  constexpr size_t kChunk = size_t(2) << 20;
  size_t pos = 0;
  for (int i = 0; i < n; ++i) {
    if (lens[i] && !chunks[i]) {
      g_err = "null chunk";
      return PLATO_INGEST_EINVAL;
    }
    if (lens[i] > dst_len - pos) {
      g_err = "chunks longer than the destination";
      return PLATO_INGEST_ECAPACITY;
    }
    for (size_t o = 0; o < lens[i]; o += kChunk)
      pieces.push_back({chunks[i] + o, dst + pos + o, std::min(kChunk, lens[i] - o)});
    pos += lens[i];
  }
  int nt = threads > 0 ? threads : int(std::max(1u, std::thread::hardware_concurrency()));
  nt = int(std::min<size_t>(size_t(nt), std::max<size_t>(1, pos / (size_t(4) << 20))));
  nt = std::min(nt, 16);
  if (nt <= 1 || pieces.size() <= 1) {
    for (auto& p : pieces) std::memcpy(p.dst, p.src, p.bytes);
  } else {
    Pool::get().run(pieces.size(), nt,
                    [&](size_t k) { std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].bytes); });
  }
  g_err.clear();
  return 0;
}

int plato_ingest_pack(const void* const* src, const uint64_t* bytes, const uint64_t* dst_off, int n, void* dst,
                      size_t dst_len, int threads) {
  if (n < 0 || (n > 0 && (!src || !bytes || !dst_off)) || (!dst && dst_len)) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  uint8_t* out = static_cast<uint8_t*>(dst);
  std::vector<Piece> pieces;
  constexpr size_t kChunk = size_t(1) << 20;
  size_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] && !src[i]) {
      g_err = "null source";
      return PLATO_INGEST_EINVAL;
    }
    if (dst_off[i] > dst_len || bytes[i] > dst_len - dst_off[i]) {
      g_err = "piece outside the destination";
      return PLATO_INGEST_ECAPACITY;
    }
    const uint8_t* from = static_cast<const uint8_t*>(src[i]);
    for (size_t o = 0; o < bytes[i]; o += kChunk)
      pieces.push_back({from + o, out + dst_off[i] + o, std::min<size_t>(kChunk, bytes[i] - o)});
    total += bytes[i];
  }
  int nt = threads > 0 ? threads : int(std::max(1u, std::thread::hardware_concurrency()));
  nt = int(std::min<size_t>(size_t(nt), std::max<size_t>(1, total / (size_t(2) << 20))));
  nt = std::min(nt, 16);
  if (nt <= 1 || pieces.size() <= 1) {
    for (auto& p : pieces) std::memcpy(p.dst, p.src, p.bytes);
  } else {
    Pool::get().run(pieces.size(), nt,
                    [&](size_t k) { std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].bytes); });
  }
  g_err.clear();
  return 0;
}

int64_t plato_ingest_read_fd(int fd, uint8_t* dst, size_t len, int threads) {
  if (fd < 0 || (!dst && len)) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  constexpr size_t kChunk = size_t(4) << 20;
  const size_t n_pieces = (len + kChunk - 1) / kChunk;
  std::atomic<int> failed{0};
  auto read_piece = [&](size_t k) {
    const size_t off = k * kChunk, want = std::min(kChunk, len - off);
    size_t got = 0;
    while (got < want) {
      const ssize_t r = ::pread(fd, dst + off + got, want - got, off_t(off + got));
      if (r > 0) {
        got += size_t(r);
      } else if (r < 0 && errno == EINTR) {
        continue;
      } else {  // error, or the file ended before len
        failed.store(r < 0 ? errno : -1);
        return;
      }
    }
  };
  int nt = threads > 0 ? threads : int(std::max(1u, std::thread::hardware_concurrency()));
  nt = std::min({nt, 16, int(std::max<size_t>(1, n_pieces))});
  if (nt <= 1) {
    for (size_t k = 0; k < n_pieces; ++k) read_piece(k);
  } else {
    Pool::get().run(n_pieces, nt, read_piece);
  }
  if (const int e = failed.load()) {
    g_err = e > 0 ? std::string("read: ") + std::strerror(e) : std::string("file shorter than expected");
    return PLATO_INGEST_EIO;
  }
  g_err.clear();
  return int64_t(len);
}

size_t plato_ingest_zstd_bound(size_t len) {
  const Zstd* z = zstd_or_fail();
  return z ? z->bound(len) : 0;
}

int64_t plato_ingest_zstd_compress(const uint8_t* src, size_t len, uint8_t* dst, size_t cap, int level) {
  const Zstd* z = zstd_or_fail();
  if (!z) return PLATO_INGEST_ENOCODEC;
  if ((len && !src) || !dst) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  const size_t r = z->compress(dst, cap, src, len, level);
  if (z->is_error(r)) {
    g_err = std::string("zstd: ") + z->error_name(r);
    return PLATO_INGEST_ECAPACITY;
  }
  g_err.clear();
  return int64_t(r);
}

int plato_ingest_parse(const uint8_t* buf, size_t len, plato_ingest_tensor* out, int max_tensors) {
  if (!buf || max_tensors < 0 || (max_tensors > 0 && !out)) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  try {
    Ctx c{buf, len, {}, {}};
    Reader r{c, 0, len};
    P top = run(c, r, nullptr);
    if (top->k != K::Dict) fail(PLATO_INGEST_EUNSUPPORTED, "payload is not a dict of tensors");
    if (int64_t(top->dict.size()) > max_tensors) {  // not an exception: a C++ throw from a library loaded
      g_err = "more tensors than the output array";  // beside torch's costs ~20 ms of FDE lookups
      return PLATO_INGEST_ECAPACITY;
    }
    int n = 0;
    for (auto& kv : top->dict) {
      if (kv.first->k != K::Str) fail(PLATO_INGEST_EUNSUPPORTED, "non-string key");
      if (kv.second->k != K::Tensor) fail(PLATO_INGEST_EUNSUPPORTED, "value is not a tensor: " + c.str(*kv.first));
      plato_ingest_tensor t = c.tensors[size_t(kv.second->i)];
      const Storage& s = c.storages[size_t(t.storage_id)];
      t.data_offset = s.data_offset;
      t.name_offset = kv.first->off;
      t.name_len = uint32_t(kv.first->len);
      out[n++] = t;
    }
    g_err.clear();
    return n;
  } catch (const Error& e) {
    g_err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    g_err = e.what();
    return PLATO_INGEST_EFORMAT;
  }
}

int plato_ingest_gather(const uint8_t* buf, size_t len, const plato_ingest_tensor* t, int n,
                        const uint64_t* dst_byte_offset, uint8_t* dst, size_t dst_len, int threads) {
  if (!buf || (n > 0 && (!t || !dst_byte_offset || !dst)) || n < 0) {
    g_err = "bad argument";
    return PLATO_INGEST_EINVAL;
  }
  std::vector<Piece> pieces;
  std::vector<int> strided;
  constexpr size_t kChunk = size_t(2) << 20;
  for (int i = 0; i < n; ++i) {
    const plato_ingest_tensor& x = t[i];
    const size_t es = size_t(x.element_size);
    const size_t bytes = size_t(x.numel) * es;
    uint64_t storage_bytes = 0;
    if (es == 0 || es > 16 || !tensor_in_storage(x) || __builtin_mul_overflow(x.storage_numel, es, &storage_bytes) ||
        x.data_offset > len || storage_bytes > len - x.data_offset || dst_byte_offset[i] > dst_len ||
        bytes > dst_len - dst_byte_offset[i]) {
      g_err = "tensor or destination out of range";
      return PLATO_INGEST_EINVAL;
    }
    if (!x.contiguous) {
      strided.push_back(i);
      continue;
    }
    const uint8_t* src = buf + x.data_offset + x.storage_offset * es;
    uint8_t* d = dst + dst_byte_offset[i];
    for (size_t o = 0; o < bytes; o += kChunk) pieces.push_back({src + o, d + o, std::min(kChunk, bytes - o)});
  }
  size_t total = 0;
  for (auto& p : pieces) total += p.bytes;
  int nt = threads > 0 ? threads : int(std::max(1u, std::thread::hardware_concurrency()));
  nt = int(std::min<size_t>(size_t(nt), std::max<size_t>(1, total / (size_t(4) << 20))));
  nt = std::min(nt, 16);
  if (nt <= 1 || pieces.size() <= 1) {
    for (auto& p : pieces) std::memcpy(p.dst, p.src, p.bytes);
  } else {
    Pool::get().run(pieces.size(), nt,
                    [&](size_t k) { std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].bytes); });
  }
  for (int i : strided) copy_strided(buf + t[i].data_offset, t[i], dst + dst_byte_offset[i]);
  g_err.clear();
  return 0;
}

}  // extern "C"
