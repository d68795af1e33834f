// qf_io.cpp — host-side TREC run I/O for the fusion path (C++17, OpenMP).
//
// Replaces the text steps around the device kernels:
//   load_runs          src/fusion.py:46-76   (pandas read_csv of every *.norm.res,
//                                             sep=r"\s+", qid/docno as str)
//   + the packing the device path needs (qppfuse/runset.py: sorted qids, docnos
//     interned in string order, CSR of (query, run) lists in file row order,
//     int32 micro-units when every score is a 6-decimal number)
//   write_runfile      src/fusion.py:480-492 ("{qid} Q0 {docno} {rank} {score:.6f}
//                                             {tag}\n", queries in the caller's
//                                             order, documents as ranked)
// Parsing is chunked over threads at line boundaries of memory-mapped files;
// strings are interned by hash partitions deduplicated in parallel, then only
// the distinct strings are sorted (byte order == Python's str order).  "%.6f" is
// Python's correctly rounded formatting: the exact binary value decides, ties
// to even — done in integers (micro-units, fma sign tests as the device's
// round6) for |x| < 2^33 and by snprintf (glibc, also exact) otherwise.
#include <emmintrin.h>
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <parallel/algorithm>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/qfio.h"

namespace {

thread_local std::string g_err;

// QFIO_TIMING=1: phase times of qfio_load_runs on stderr (diagnostics).
struct PhaseTimer {
  bool on = getenv("QFIO_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[qfio] %-18s %8.3f ms\n", what,
            std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct Mapped {
  const char* data = nullptr;
  size_t size = 0;
  int fd = -1;
  ~Mapped() {
    if (data && size) munmap((void*)data, size);
    if (fd >= 0) close(fd);
  }
};


// A column buffer that is NOT initialised on allocation (the parse writes every
// element, in parallel, so the pages are first touched by the threads that fill
// them); large ones are anonymous mappings with transparent huge pages asked for.
template <class T>
struct RawArray {
  T* a = nullptr;
  size_t n = 0, bytes = 0;
  bool mapped = false;
  RawArray() = default;
  RawArray(const RawArray&) = delete;
  RawArray& operator=(const RawArray&) = delete;
  RawArray(RawArray&& o) noexcept { *this = std::move(o); }
  RawArray& operator=(RawArray&& o) noexcept {
    if (this != &o) {
      release();
      a = o.a; n = o.n; bytes = o.bytes; mapped = o.mapped;
      o.a = nullptr; o.n = o.bytes = 0; o.mapped = false;
    }
    return *this;
  }
  ~RawArray() { release(); }
  void release() {
    if (a && mapped) munmap((void*)a, bytes);
    else free(a);
    a = nullptr;
    n = bytes = 0;
    mapped = false;  // a later small resize() mallocs: never munmap that
  }
  void resize(size_t m) {  // contents undefined
    release();
    n = m;
    bytes = std::max<size_t>(1, m * sizeof(T));
    if (bytes >= (size_t)4 << 20) {
      void* v = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (v != MAP_FAILED) {
        madvise(v, bytes, MADV_HUGEPAGE);
        a = (T*)v;
        mapped = true;
        return;
      }
    }
    a = (T*)malloc(bytes);
    if (!a) throw std::bad_alloc();
  }
  // hands a mapped buffer to `bin` (to be unmapped later), frees a small one now
  void release_to(std::vector<std::pair<void*, size_t>>& bin) {
    if (a && mapped) bin.emplace_back((void*)a, bytes);
    else free(a);
    a = nullptr;
    n = bytes = 0;
    mapped = false;
  }
  size_t size() const { return n; }
  const T* begin() const { return a; }
  const T* end() const { return a + n; }
  T& operator[](size_t i) { return a[i]; }
  const T& operator[](size_t i) const { return a[i]; }
  T* data() { return a; }
  const T* data() const { return a; }
};

// Gives back the buffers of large temporaries on a thread of its own: freeing a few
// hundred MB of touched pages costs tens of ms that need not be on the caller's
// path.  The pages go first (madvise takes the address-space lock shared, so the
// caller's page faults proceed meanwhile); the munmap, which takes it exclusively,
// then has nothing left to free.
template <class... A>
void release_async(A&... arrays) {
  auto* bin = new std::vector<std::pair<void*, size_t>>();
  (arrays.release_to(*bin), ...);
  std::thread([bin] {
    for (auto& m : *bin) madvise(m.first, m.second, MADV_DONTNEED);
    for (auto& m : *bin) munmap(m.first, m.second);
    delete bin;
  }).detach();
}

// A string view that is trivially constructible (rows of the column buffers).
struct SV {
  const char* p;
  size_t n;
};
inline std::string_view sv(const SV& v) { return std::string_view(v.p, v.n); }
inline std::string_view sv(std::string_view v) { return v; }

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }
// is_space as a table (the parse's per-byte test)
struct SpaceTable {
  bool t[256];
  constexpr SpaceTable() : t{} {
    t[(unsigned char)' '] = t[(unsigned char)'\t'] = t[(unsigned char)'\r'] = true;
    t[(unsigned char)'\v'] = t[(unsigned char)'\f'] = true;
  }
  constexpr bool operator[](unsigned char c) const { return t[c]; }
};
constexpr SpaceTable kSpace{};

// [-]digits[.digits<=6] that fits int32 micro-units; "-0.000000" (which parses
// to -0.0) is excluded.
inline bool micro_text(std::string_view t, int32_t& micro) {
  size_t i = 0;
  bool neg = false;
  if (i < t.size() && (t[i] == '-' || t[i] == '+')) neg = t[i++] == '-';
  int64_t ip = 0, fp = 0;
  int nd = 0, fd = 0;
  while (i < t.size() && t[i] >= '0' && t[i] <= '9' && nd < 12) { ip = ip * 10 + (t[i++] - '0'); ++nd; }
  if (nd == 0) return false;
  if (i < t.size() && t[i] == '.') {
    ++i;
    while (i < t.size() && t[i] >= '0' && t[i] <= '9' && fd < 7) { fp = fp * 10 + (t[i++] - '0'); ++fd; }
  }
  if (i != t.size() || fd > 6) return false;
  for (int k = fd; k < 6; ++k) fp *= 10;
  const int64_t m = ip * 1000000 + fp;
  if (m >= 2147483647LL || (neg && m == 0)) return false;
  micro = (int32_t)(neg ? -m : m);
  return true;
}

// pandas/CPython float text -> double (correctly rounded, strtod) and, when the
// text is [-]digits[.digits<=6], its exact micro-unit integer.
inline bool parse_score(std::string_view t, double& v, int32_t& micro, bool& micro_ok) {
  micro_ok = false;
  if (micro_text(t, micro)) {  // m / 1e6 is the correctly rounded value of the text too
    v = (double)micro / 1e6;
    micro_ok = true;
    return true;
  }
  char buf[64];
  if (t.size() >= sizeof buf) return false;
  memcpy(buf, t.data(), t.size());
  buf[t.size()] = 0;
  char* end = nullptr;
  errno = 0;
  v = strtod(buf, &end);
  return end == buf + t.size();
}

// Rows with any non-blank field in [p, end) (pandas skips blank lines).
size_t count_rows(const char* p, const char* end) {
  size_t n = 0;
  while (p < end) {
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* e = nl ? nl : end;
    const char* q = p;
    while (q < e && (is_space(*q))) ++q;
    n += q < e;
    p = nl ? nl + 1 : end;
  }
  return n;
}

inline uint64_t hash_sv(std::string_view v) {  // FNV-1a + avalanche
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : v) h = (h ^ c) * 1099511628211ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

// The parse's docno hash (consistent within one load; intern() partitions and
// probes by it): 8 bytes per multiply instead of FNV's one.
inline uint64_t hash_words(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    h = (h ^ w) * 0xff51afd7ed558ccdull;
    h ^= h >> 32;
  }
  if (i < n) {
    uint64_t w = 0;
    memcpy(&w, p + i, n - i);
    h = (h ^ w) * 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 29;
  }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

// Whitespace bytes (' ' and \t \n \v \f \r) of 16 bytes at p, as a bit mask.
inline uint32_t ws_mask16(const char* p) {
  const __m128i c = _mm_loadu_si128((const __m128i*)p);
  const __m128i sp = _mm_cmpeq_epi8(c, _mm_set1_epi8(' '));
  const __m128i x = _mm_sub_epi8(c, _mm_set1_epi8(9));
  const __m128i ctl = _mm_cmpeq_epi8(_mm_min_epu8(x, _mm_set1_epi8(4)), x);
  return (uint32_t)_mm_movemask_epi8(_mm_or_si128(sp, ctl));
}

// Row columns, structure of arrays over all files in file order.  The parse also
// hashes each docno (its bytes are in cache then).  qid / iter / tag are long runs
// of one value: only their run heads (a row whose value differs from the row
// before, or a chunk's first row) are kept, per parse chunk — 44 bytes per row
// written instead of 95 (the columns are fresh pages: every byte is a page-fault
// byte too).
struct Head {
  size_t row;
  SV v;
};
struct Heads {
  std::vector<Head> q, it, tag;
};
struct Cols {
  RawArray<SV> d;
  RawArray<int64_t> rank;
  RawArray<double> score;
  RawArray<int32_t> micro;
  RawArray<uint64_t> dh;  // docno hashes
  void resize(size_t n) {
    d.resize(n);
    rank.resize(n); score.resize(n); micro.resize(n);
    dh.resize(n);
  }
};

// Parse [begin, end) of a mapped file (whole lines) into rows o, o+1, ...;
// micro_bad_out: the number of rows whose score is not an exact 6-decimal number.
// The count is kept in a local and stored once: the per-chunk counters sit side by
// side in one vector, and a per-row store to them (the compiler must store it, the
// row columns may alias a size_t) made the threads fight over those cache lines —
// the parse ran 1.6x faster on 8 threads than on 1 (4x after the fix).
bool parse_chunk(const char* p, const char* end, const char* map_end, Cols& c, Heads& h,
                 size_t o, size_t& micro_bad_out, std::string& err) {
  size_t micro_bad = 0;
  std::string_view pq, pit, ptag;  // the previous row's (a chunk's first row is a head)
  bool first = true;
  while (p < end) {
    std::string_view f[7];
    int nf = 0;
    const char* line = p;
    // the line's end first (memchr), then the fields inside it by a table lookup
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* e = nl ? nl : end;
    const size_t len = (size_t)(e - p);
    if (len < 64 && (size_t)(map_end - p) >= 64) {
      // the fields from a whitespace bit mask of the line (16-byte loads that stay
      // inside the mapping; bits past the line count as whitespace)
      uint64_t ws = 0;
      for (size_t k = 0; k < len; k += 16) ws |= (uint64_t)ws_mask16(p + k) << k;
      ws |= ~0ull << len;
      uint64_t st = ~ws & ((ws << 1) | 1u);  // first byte of a field
      uint64_t en = ws & (~ws << 1);         // first byte after a field
      nf = __builtin_popcountll(st);
      for (int k = 0; k < nf && k < 7; ++k) {
        const int a = __builtin_ctzll(st), b = __builtin_ctzll(en);
        f[k] = std::string_view(p + a, (size_t)(b - a));
        st &= st - 1;
        en &= en - 1;
      }
    } else {
      const char* q = p;
      while (true) {
        while (q < e && kSpace[(unsigned char)*q]) ++q;
        if (q >= e) break;
        const char* s = q;
        while (q < e && !kSpace[(unsigned char)*q]) ++q;
        if (nf < 7) f[nf] = std::string_view(s, (size_t)(q - s));
        ++nf;
      }
    }
    p = nl ? nl + 1 : end;
    if (nf == 0) continue;  // blank line (pandas skips it)
    if (nf != 6) {
      err = "expected 6 fields (qid Q0 docno rank score tag), got " + std::to_string(nf) +
            " in line: " + std::string(line, std::min<size_t>(120, (size_t)(p - line)));
      return false;
    }
    c.d[o] = SV{f[2].data(), f[2].size()};
    c.dh[o] = hash_words(f[2].data(), f[2].size());
    if (first || f[0] != pq) h.q.push_back(Head{o, SV{f[0].data(), f[0].size()}});
    if (first || f[1] != pit) h.it.push_back(Head{o, SV{f[1].data(), f[1].size()}});
    if (first || f[5] != ptag) h.tag.push_back(Head{o, SV{f[5].data(), f[5].size()}});
    pq = f[0]; pit = f[1]; ptag = f[5];
    first = false;
    // rank: [+-]digits (strtoll's accepted form for plain integer text)
    {
      const std::string_view t = f[3];
      size_t i = 0;
      bool neg = false;
      if (i < t.size() && (t[i] == '-' || t[i] == '+')) neg = t[i++] == '-';
      int64_t v = 0;
      const size_t d0 = i;
      while (i < t.size() && t[i] >= '0' && t[i] <= '9' && i - d0 < 18) v = v * 10 + (t[i++] - '0');
      if (i == d0 || i != t.size()) { err = "bad rank field '" + std::string(t) + "'"; return false; }
      c.rank[o] = neg ? -v : v;
    }
    bool mok = false;
    int32_t m = 0;
    if (!parse_score(f[4], c.score[o], m, mok)) {
      err = "bad score field '" + std::string(f[4]) + "'";
      return false;
    }
    c.micro[o] = m;
    micro_bad += !mok;
    ++o;
  }
  micro_bad_out = micro_bad;
  return true;
}

// Sorted unique strings of `views`, and each view's index among them: hash
// partitions deduplicated in parallel, then only the distinct strings sorted.
// The sort key of a distinct string: its first 16 bytes big-endian, zero-padded
// (no NUL in the text, so a proper prefix sorts first); only equal keys compare
// the strings.  Sorting 24-byte records keeps the sort in cache instead of
// chasing string pointers.
struct Key {
  uint64_t k1, k2;
  uint32_t u;
};
inline void key16(std::string_view v, uint64_t& k1, uint64_t& k2) {
  unsigned char b[16] = {0};
  memcpy(b, v.data(), std::min<size_t>(16, v.size()));
  uint64_t w1, w2;
  memcpy(&w1, b, 8);
  memcpy(&w2, b + 8, 8);
  k1 = __builtin_bswap64(w1);
  k2 = __builtin_bswap64(w2);
}
// a row on its way to the dedupe, and a distinct string found there
struct PartEnt {
  uint64_t h, k1, k2;
  uint32_t row, len;
};
struct Rep {
  uint64_t h, k1, k2;
  uint32_t len, row;
};

// hs_in: the strings' hash_sv values when the caller has them (the parse's)
template <class Views>
void intern(const Views& views, RawArray<SV>& uniq, RawArray<uint32_t>& id,
            const uint64_t* hs_in = nullptr) {
  PhaseTimer tm;
  const size_t n = views.size();
  // hash partitions: 4,096 for large sets (a partition's probe table and distinct
  // strings — ~4 K rows, ~2 K strings for C2's 17 M docnos — stay in the core's
  // cache during its dedupe), 256 for small ones (the run heads)
  const int PB = n >= ((size_t)1 << 22) ? 12 : 8, P = 1 << PB, PS = 64 - PB;
  RawArray<uint64_t> hs_own;
  const uint64_t* hs = hs_in;
  if (!hs) {
    hs_own.resize(n);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < n; ++i) hs_own[i] = hash_sv(sv(views[i]));
    hs = hs_own.data();
  }
  // rows of each partition (top 8 bits), in row order
  const int T = std::max(1, omp_get_max_threads());
  std::vector<std::vector<uint32_t>> cnt(T, std::vector<uint32_t>(P, 0));
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T; ++t)
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) ++cnt[t][hs[i] >> PS];
  std::vector<size_t> start(P + 1, 0);
  for (int b = 0; b < P; ++b) {
    size_t s = 0;
    for (int t = 0; t < T; ++t) s += cnt[t][b];
    start[b + 1] = start[b] + s;
  }
  std::vector<std::vector<size_t>> at(T, std::vector<size_t>(P));
  for (int b = 0; b < P; ++b) {
    size_t o = start[b];
    for (int t = 0; t < T; ++t) { at[t][b] = o; o += cnt[t][b]; }
  }
  // Each row goes to its partition as (hash, first 16 bytes, row, length), read
  // here in row order (the text sequentially): the dedupe then streams its
  // partition and keeps, per distinct string, the same fields beside the probe
  // table — a string of <= 16 bytes is recognised from them alone, without
  // touching any row's view or text at random.  (Was: row indices only; every probe
  // fetched the row's hash, view and text, and every hit the first occurrence's.)
  RawArray<PartEnt> ents;  // uninitialised: the scatter writes every element
  ents.resize(n);
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T; ++t)
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) {
      const std::string_view v = sv(views[i]);
      uint64_t k1, k2;
      key16(v, k1, k2);
      ents[at[t][hs[i] >> PS]++] = PartEnt{hs[i], k1, k2, (uint32_t)i, (uint32_t)v.size()};
    }
  tm.mark("  hash+partition");
  // per partition: open-addressing table -> local unique index
  std::vector<std::vector<Rep>> urep(P);
  RawArray<uint32_t> local;
  local.resize(n);
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < P; ++b) {
    const size_t a0 = start[b], a1 = start[b + 1], m = a1 - a0;
    if (!m) continue;
    size_t cap = 16;
    while (cap < 2 * m) cap <<= 1;
    std::vector<uint32_t> tab(cap, 0xFFFFFFFFu);
    // built locally and moved in at the end (the vector headers in urep share
    // cache lines with the neighbouring partitions')
    std::vector<Rep> rep;
    rep.reserve(m);  // at most m distinct: no regrowth copies
    for (size_t k = a0; k < a1; ++k) {
      const PartEnt e = ents[k];
      size_t h = (size_t)e.h & (cap - 1);
      while (true) {
        const uint32_t u = tab[h];
        if (u == 0xFFFFFFFFu) {
          tab[h] = (uint32_t)rep.size();
          local[e.row] = (uint32_t)rep.size();
          rep.push_back(Rep{e.h, e.k1, e.k2, e.len, e.row});
          break;
        }
        const Rep& r = rep[u];
        if (r.h == e.h && r.len == e.len && r.k1 == e.k1 && r.k2 == e.k2 &&
            (e.len <= 16 || memcmp(sv(views[r.row]).data() + 16, sv(views[e.row]).data() + 16,
                                   e.len - 16) == 0)) {
          local[e.row] = u;
          break;
        }
        h = (h + 1) & (cap - 1);
      }
    }
    urep[b] = std::move(rep);
  }
  tm.mark("  dedupe");
  std::vector<size_t> ubase(P + 1, 0);
  for (int b = 0; b < P; ++b) ubase[b + 1] = ubase[b] + urep[b].size();
  const size_t U = ubase[P];
  RawArray<uint32_t> reps;  // row of each distinct string
  RawArray<Key> keys;
  reps.resize(U);
  keys.resize(U);
  // Sort the distinct strings by byte order (== Python's str order for UTF-8).
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < P; ++b) {
    const std::vector<Rep>& rep = urep[b];
    for (size_t j = 0; j < rep.size(); ++j) {
      reps[ubase[b] + j] = rep[j].row;
      keys[ubase[b] + j] = Key{rep[j].k1, rep[j].k2, (uint32_t)(ubase[b] + j)};
    }
  }
  auto less = [&](const Key& a, const Key& b) {
    if (a.k1 != b.k1) return a.k1 < b.k1;
    if (a.k2 != b.k2) return a.k2 < b.k2;
    return sv(views[reps[a.u]]) < sv(views[reps[b.u]]);
  };
  tm.mark("  keys");
  // (Measured, not kept: sampled range buckets — 4,096 splitters, a binary search
  // per key, a counting scatter, per-bucket sorts — 115 ms on the GPU box's host
  // against the parallel sort's ~65 ms for C2's 8.6 M distinct docnos.)
  __gnu_parallel::sort(keys.data(), keys.data() + U, less);
  tm.mark("  sort distinct");
  RawArray<uint32_t> rank;
  rank.resize(U);
  uniq.resize(U);
#pragma omp parallel for schedule(static)
  for (size_t k = 0; k < U; ++k) {
    if (k + 16 < U) __builtin_prefetch(&views[reps[keys[k + 16].u]]);
    rank[keys[k].u] = (uint32_t)k;
    const std::string_view v = sv(views[reps[keys[k].u]]);
    uniq[k] = SV{v.data(), v.size()};
  }
  id.resize(n);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) {
    if (i + 16 < n) __builtin_prefetch(&rank[ubase[hs[i + 16] >> PS] + local[i + 16]]);
    id[i] = rank[ubase[hs[i] >> PS] + local[i]];
  }
  tm.mark("  ranks");
  release_async(hs_own, ents, local, reps, keys, rank);
}

// intern() for columns made of long runs of one value (qid, Q0, tag): only the
// run heads the parse kept are interned (a head too many — a chunk's first row —
// costs one more string), then every row takes its run's id.
// head_rows / head_ids (optional): the runs (first row, id), in row order.
void intern_runs(const std::vector<Heads>& heads, std::vector<Head> Heads::*which, size_t n,
                 RawArray<SV>& uniq, RawArray<uint32_t>& id,
                 std::vector<size_t>* head_rows = nullptr, RawArray<uint32_t>* head_ids = nullptr) {
  std::vector<size_t> hix;
  std::vector<std::string_view> hv;
  size_t nh = 0;
  for (const Heads& h : heads) nh += (h.*which).size();
  hix.reserve(nh);
  hv.reserve(nh);
  for (const Heads& h : heads)  // chunks in row order
    for (const Head& x : h.*which) {
      hix.push_back(x.row);
      hv.push_back(sv(x.v));
    }
  RawArray<uint32_t> hid;
  intern(hv, uniq, hid);
  id.resize(n);
#pragma omp parallel for schedule(dynamic, 64)
  for (size_t k = 0; k < hix.size(); ++k) {
    const size_t e = k + 1 < hix.size() ? hix[k + 1] : n;
    for (size_t i = hix[k]; i < e; ++i) id[i] = hid[k];
  }
  if (head_rows) *head_rows = std::move(hix);
  if (head_ids) *head_ids = std::move(hid);
}

}  // namespace

struct qfio_runset {
  std::vector<Mapped*> maps;
  int32_t n_files = 0;
  // the distinct strings in byte order (views into the mapped files; RawArrays:
  // no serial zero-fill of C2's 8.6 M docno views)
  RawArray<SV> qids, docnos, iters, tags;
  // CSR (query-major, run-minor), rows in file order
  std::vector<int64_t> list_off;
  RawArray<uint32_t> docid;
  RawArray<double> score;
  RawArray<int32_t> micro;
  RawArray<int64_t> rank;
  bool micro_ok = true;
  bool rank_is_position = true, canonical = true, has_dups = false;
  // per-file rows in file order (for DataFrames): codes and values
  std::vector<int64_t> file_off;  // [n_files + 1]
  RawArray<uint32_t> row_qid, row_docid, row_iter, row_tag;
  RawArray<int64_t> row_rank;
  RawArray<double> row_score;
  ~qfio_runset() {
    for (auto* m : maps) delete m;
  }
};

// memcpy over the threads (the column copies out of the run set are 0.1-0.3 GB)
static void pcopy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kChunk = (size_t)8 << 20;
  const int64_t nc = (int64_t)((bytes + kChunk - 1) / kChunk);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t c = 0; c < nc; ++c) {
    const size_t a = (size_t)c * kChunk, e = std::min(bytes, a + kChunk);
    memcpy((char*)dst + a, (const char*)src + a, e - a);
  }
}

extern "C" {

const char* qfio_last_error(void) { return g_err.c_str(); }

int qfio_load_runs(const char* const* paths, int32_t n_files, int32_t n_threads,
                   qfio_runset** out) {
  if (!paths || n_files <= 0 || !out) return fail(QFIO_EINVAL, "qfio_load_runs: bad arguments");
  if (n_threads > 0) omp_set_num_threads(n_threads);
  auto* rs = new qfio_runset();
  rs->n_files = n_files;
  PhaseTimer tm;
  // ---- map every file; chunk at line boundaries; count rows per chunk ----------
  const int T = std::max(1, omp_get_max_threads());
  std::vector<const char*> cut((size_t)n_files * (T + 1));
  for (int f = 0; f < n_files; ++f) {
    auto* m = new Mapped();
    rs->maps.push_back(m);
    m->fd = open(paths[f], O_RDONLY);
    if (m->fd < 0) {
      delete rs;
      return fail(QFIO_ENOENT, std::string("cannot open ") + paths[f] + ": " + strerror(errno));
    }
    struct stat st;
    fstat(m->fd, &st);
    m->size = (size_t)st.st_size;
    if (m->size) {
      m->data = (const char*)mmap(nullptr, m->size, PROT_READ, MAP_PRIVATE | MAP_POPULATE,
                                  m->fd, 0);
      if (m->data == MAP_FAILED) {
        m->data = nullptr;
        delete rs;
        return fail(QFIO_EIO, std::string("cannot map ") + paths[f]);
      }
    }
    const char** c = &cut[(size_t)f * (T + 1)];
    c[0] = m->data;
    c[T] = m->data + m->size;
    for (int t = 1; t < T; ++t) {
      const char* x = m->data + (m->size * (size_t)t) / (size_t)T;
      while (x < c[T] && x > m->data && x[-1] != '\n') ++x;
      c[t] = std::max(x, c[t - 1]);
    }
  }
  tm.mark("map");
  const size_t NC = (size_t)n_files * T;
  std::vector<size_t> nrow(NC + 1, 0);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t k = 0; k < NC; ++k) {
    const size_t f = k / T, t = k % T;
    nrow[k + 1] = count_rows(cut[f * (T + 1) + t], cut[f * (T + 1) + t + 1]);
  }
  for (size_t k = 0; k < NC; ++k) nrow[k + 1] += nrow[k];
  const size_t E = nrow[NC];
  if (E >= 0xFFFFFFFFull) { delete rs; return fail(QFIO_EINVAL, "too many rows"); }
  rs->file_off.assign(n_files + 1, 0);
  for (int f = 0; f <= n_files; ++f) rs->file_off[f] = (int64_t)nrow[(size_t)f * T];
  // ---- parse every chunk straight into its rows ------------------------------
  tm.mark("count rows");
  Cols cols;
  cols.resize(E);
  tm.mark("alloc columns");
  std::vector<std::string> errs(NC);
  std::vector<size_t> mbad(NC, 0);
  std::vector<Heads> heads(NC);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t k = 0; k < NC; ++k) {
    const size_t f = k / T, t = k % T;
    parse_chunk(cut[f * (T + 1) + t], cut[f * (T + 1) + t + 1], cut[f * (T + 1) + T], cols, heads[k],
                nrow[k], mbad[k], errs[k]);
  }
  tm.mark("parse");
  for (size_t k = 0; k < NC; ++k)
    if (!errs[k].empty()) {
      const std::string e = std::string(paths[k / T]) + ": " + errs[k];
      delete rs;
      return fail(QFIO_EPARSE, e);
    }
  size_t micro_bad = 0;
  for (size_t k = 0; k < NC; ++k) micro_bad += mbad[k];
  rs->micro_ok = micro_bad == 0;
  rs->row_rank = std::move(cols.rank);
  rs->row_score = std::move(cols.score);
  RawArray<int32_t> row_micro = std::move(cols.micro);
  // ---- intern qids / docnos / iter / tag ---------------------------------------
  std::vector<size_t> qrun_row;  // runs of one qid (no run crosses a file: a file's
  RawArray<uint32_t> qrun_id;    // first row starts a parse chunk, hence a run)
  intern_runs(heads, &Heads::q, E, rs->qids, rs->row_qid, &qrun_row, &qrun_id);
  tm.mark("intern qid");
  intern(cols.d, rs->docnos, rs->row_docid, cols.dh.data());
  tm.mark("intern docno");
  intern_runs(heads, &Heads::it, E, rs->iters, rs->row_iter);
  intern_runs(heads, &Heads::tag, E, rs->tags, rs->row_tag);
  tm.mark("intern iter/tag");
  if (rs->docnos.size() >= 0xFFFFFFFFull) { delete rs; return fail(QFIO_EINVAL, "too many docnos"); }
  // ---- CSR by (query, file), stable in file order -------------------------------
  // from the qid runs: counts per list, each run's destination in run (= row)
  // order, then the runs copied in parallel
  const int64_t Q = (int64_t)rs->qids.size(), R = n_files;
  const size_t NR = qrun_row.size();
  std::vector<int64_t> rlist(NR), rlen(NR), rdst(NR);
  std::vector<int64_t> cnt(Q * R + 1, 0);
  {
    int f = 0;
    for (size_t k = 0; k < NR; ++k) {
      const int64_t a = (int64_t)qrun_row[k], e = k + 1 < NR ? (int64_t)qrun_row[k + 1] : (int64_t)E;
      while (a >= rs->file_off[f + 1]) ++f;
      rlist[k] = (int64_t)qrun_id[k] * R + f;
      rlen[k] = e - a;
      cnt[rlist[k]] += rlen[k];
    }
  }
  rs->list_off.assign(Q * R + 1, 0);
  for (int64_t k = 0; k < Q * R; ++k) rs->list_off[k + 1] = rs->list_off[k] + cnt[k];
  {
    std::vector<int64_t> pos(rs->list_off.begin(), rs->list_off.end() - 1);
    for (size_t k = 0; k < NR; ++k) {
      rdst[k] = pos[rlist[k]];
      pos[rlist[k]] += rlen[k];
    }
  }
  rs->docid.resize(E);
  rs->score.resize(E);
  rs->rank.resize(E);
  rs->micro.resize(rs->micro_ok ? E : 0);
#pragma omp parallel for schedule(dynamic, 16)
  for (size_t k = 0; k < NR; ++k) {
    const int64_t a = (int64_t)qrun_row[k], d = rdst[k], n = rlen[k];
    memcpy(&rs->docid[d], &rs->row_docid[a], (size_t)n * sizeof(uint32_t));
    memcpy(&rs->score[d], &rs->row_score[a], (size_t)n * sizeof(double));
    memcpy(&rs->rank[d], &rs->row_rank[a], (size_t)n * sizeof(int64_t));
    if (rs->micro_ok) memcpy(&rs->micro[d], &row_micro[a], (size_t)n * sizeof(int32_t));
  }
  // list properties the device path keys on (qppfuse/runset.py _analyse): the
  // rank column is position + 1; every list is score-descending with rising ranks
  // and whether a docno repeats inside one list (open addressing per list)
  int not_pos = 0, not_canon = 0, dups = 0;
#pragma omp parallel reduction(+ : not_pos, not_canon, dups)
  {
    std::vector<uint32_t> table;
#pragma omp for schedule(static)
    for (int64_t l = 0; l < Q * R; ++l) {
      const int64_t a = rs->list_off[l], b = rs->list_off[l + 1];
      for (int64_t i = a; i < b; ++i) {
        not_pos += rs->rank[i] != i - a + 1;
        if (i > a) not_canon += !(rs->score[i] <= rs->score[i - 1] && rs->rank[i] > rs->rank[i - 1]);
      }
      if (b - a < 2) continue;
      size_t ts = 4;
      while (ts < 2 * (size_t)(b - a)) ts <<= 1;
      table.assign(ts, 0xFFFFFFFFu);
      for (int64_t i = a; i < b; ++i) {
        const uint32_t d = rs->docid[i];
        size_t h = (size_t)((d * 0x9E3779B1u) & (uint32_t)(ts - 1));
        while (table[h] != 0xFFFFFFFFu && table[h] != d) h = (h + 1) & (ts - 1);
        if (table[h] == d) { ++dups; break; }
        table[h] = d;
      }
    }
  }
  rs->rank_is_position = not_pos == 0;
  rs->canonical = not_canon == 0;
  rs->has_dups = dups != 0;
  tm.mark("csr");
  // the per-row views and hashes (~0.4 GB for C2) go on a thread of their own
  release_async(cols.d, cols.dh, cols.rank, cols.score, cols.micro, row_micro);
  tm.mark("release columns");
  *out = rs;
  return QFIO_OK;
}

void qfio_runset_sizes(const qfio_runset* rs, int64_t* sizes /* [8] */) {
  int64_t qb = 0, db = 0, ib = 0, tb = 0;
  for (auto& s : rs->qids) qb += (int64_t)s.n;
  for (auto& s : rs->docnos) db += (int64_t)s.n;
  for (auto& s : rs->iters) ib += (int64_t)s.n;
  for (auto& s : rs->tags) tb += (int64_t)s.n;
  sizes[0] = (int64_t)rs->qids.size();
  sizes[1] = (int64_t)rs->docnos.size();
  sizes[2] = (int64_t)rs->docid.size();
  sizes[3] = qb;
  sizes[4] = db;
  sizes[5] = (rs->micro_ok ? 1 : 0) | (rs->rank_is_position ? 2 : 0) | (rs->canonical ? 4 : 0) |
             (rs->has_dups ? 8 : 0);
  sizes[6] = (int64_t)rs->iters.size() | ((int64_t)rs->tags.size() << 32);
  sizes[7] = ib | (tb << 32);
}

static void copy_strings(const RawArray<SV>& v, int64_t* off, char* chars) {
  // offsets: a blocked parallel scan (the 69 MB of C2's docno offsets are fresh pages)
  const int64_t n = (int64_t)v.size();
  off[0] = 0;
  const int T = std::max(1, omp_get_max_threads());
  std::vector<int64_t> part((size_t)T + 1, 0);
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t a = n * t / nt, b = n * (t + 1) / nt;
    int64_t o = 0;
    for (int64_t i = a; i < b; ++i) {
      o += (int64_t)v[(size_t)i].n;
      off[i + 1] = o;
    }
    part[(size_t)t + 1] = o;
#pragma omp barrier
#pragma omp single
    for (int k = 0; k < nt; ++k) part[(size_t)k + 1] += part[(size_t)k];
    const int64_t add = part[(size_t)t];
    for (int64_t i = a; i < b; ++i) off[i + 1] += add;
  }
  // the bytes in parallel: the views point all over the mapped files
#pragma omp parallel for schedule(static, 4096)
  for (int64_t i = 0; i < (int64_t)v.size(); ++i) {
    if (i + 8 < (int64_t)v.size()) __builtin_prefetch(v[i + 8].p);
    memcpy(chars + off[i], v[i].p, v[i].n);
  }
}

int qfio_runset_csr(const qfio_runset* rs, int64_t* list_off, uint32_t* docid, double* score,
                    int32_t* micro, int64_t* rank) {
  memcpy(list_off, rs->list_off.data(), rs->list_off.size() * sizeof(int64_t));
  pcopy(docid, rs->docid.data(), rs->docid.size() * sizeof(uint32_t));
  pcopy(score, rs->score.data(), rs->score.size() * sizeof(double));
  pcopy(rank, rs->rank.data(), rs->rank.size() * sizeof(int64_t));
  if (micro && rs->micro_ok) pcopy(micro, rs->micro.data(), rs->micro.size() * sizeof(int32_t));
  return QFIO_OK;
}

int qfio_runset_strings(const qfio_runset* rs, int64_t* qid_off, char* qid_chars,
                        int64_t* docno_off, char* docno_chars, int64_t* iter_off,
                        char* iter_chars, int64_t* tag_off, char* tag_chars) {
  copy_strings(rs->qids, qid_off, qid_chars);
  copy_strings(rs->docnos, docno_off, docno_chars);
  copy_strings(rs->iters, iter_off, iter_chars);
  copy_strings(rs->tags, tag_off, tag_chars);
  return QFIO_OK;
}

int qfio_join_lines(const int64_t* off, const char* chars, int64_t n, char* out) {
  if (n < 0 || (n > 0 && (!off || !chars || !out))) return fail(QFIO_EINVAL, "qfio_join_lines: bad arguments");
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = off[i], len = off[i + 1] - a;
    memcpy(out + a + i, chars + a, (size_t)len);
    out[a + i + len] = '\n';
  }
  return QFIO_OK;
}

int qfio_runset_rows(const qfio_runset* rs, int64_t* file_off, uint32_t* qid, uint32_t* docid,
                     uint32_t* iter, uint32_t* tag, int64_t* rank, double* score) {
  const size_t E = rs->row_qid.size();
  memcpy(file_off, rs->file_off.data(), rs->file_off.size() * sizeof(int64_t));
  pcopy(qid, rs->row_qid.data(), E * sizeof(uint32_t));
  pcopy(docid, rs->row_docid.data(), E * sizeof(uint32_t));
  pcopy(iter, rs->row_iter.data(), E * sizeof(uint32_t));
  pcopy(tag, rs->row_tag.data(), E * sizeof(uint32_t));
  pcopy(rank, rs->row_rank.data(), E * sizeof(int64_t));
  pcopy(score, rs->row_score.data(), E * sizeof(double));
  return QFIO_OK;
}

void qfio_runset_drop_text(qfio_runset* rs) {
  rs->qids.release();
  rs->docnos.release();
  rs->iters.release();
  rs->tags.release();
  for (auto* m : rs->maps) delete m;
  rs->maps.clear();
}

void qfio_runset_views(const qfio_runset* rs, const void** ptrs) {
  ptrs[0] = rs->list_off.data();
  ptrs[1] = rs->docid.data();
  ptrs[2] = rs->score.data();
  ptrs[3] = rs->micro_ok ? rs->micro.data() : nullptr;
  ptrs[4] = rs->rank.data();
  ptrs[5] = rs->file_off.data();
  ptrs[6] = rs->row_qid.data();
  ptrs[7] = rs->row_docid.data();
  ptrs[8] = rs->row_iter.data();
  ptrs[9] = rs->row_tag.data();
  ptrs[10] = rs->row_rank.data();
  ptrs[11] = rs->row_score.data();
}

}  // extern "C"
template <class Off>
static int64_t gather_strings(const int64_t* tab_off, const char* tab_chars, const uint32_t* codes,
                              int64_t n, Off* out_off, char* out_chars) {
  if (n < 0 || !tab_off || (n && (!codes || !out_off))) return -1;
  // lengths -> offsets (a blocked parallel scan), then the bytes
  const int T = std::max(1, omp_get_max_threads());
  std::vector<int64_t> part(T + 1, 0);
  out_off[0] = 0;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const int64_t a = n * t / nt, b = n * (t + 1) / nt;
    int64_t s = 0;
    for (int64_t i = a; i < b; ++i) {
      // a docno column's codes jump over a table far larger than the caches
      if (i + 16 < b) __builtin_prefetch(&tab_off[codes[i + 16]]);
      s += tab_off[codes[i] + 1] - tab_off[codes[i]];
      out_off[i + 1] = (Off)s;
    }
    part[t + 1] = s;
#pragma omp barrier
#pragma omp single
    for (int k = 0; k < nt; ++k) part[k + 1] += part[k];
    const int64_t add = part[t];
    for (int64_t i = a; i < b; ++i) out_off[i + 1] += (Off)add;
#pragma omp barrier  // out_off[a] is the previous thread's last offset
    if (out_chars)
      for (int64_t i = a; i < b; ++i) {
        if (i + 16 < b) __builtin_prefetch(&tab_off[codes[i + 16]]);
        if (i + 8 < b) __builtin_prefetch(tab_chars + tab_off[codes[i + 8]]);
        memcpy(out_chars + out_off[i], tab_chars + tab_off[codes[i]],
               (size_t)(out_off[i + 1] - out_off[i]));
      }
  }
  return n ? (int64_t)out_off[n] : 0;
}
extern "C" {

int64_t qfio_gather_strings(const int64_t* tab_off, const char* tab_chars, const uint32_t* codes,
                            int64_t n, int64_t* out_off, char* out_chars) {
  return gather_strings(tab_off, tab_chars, codes, n, out_off, out_chars);
}

int qfio_gather_chars(const int64_t* tab_off, const char* tab_chars, const uint32_t* codes,
                      int64_t n, const int64_t* out_off, char* out_chars) {
  if (n < 0 || (n && (!tab_off || !tab_chars || !codes || !out_off || !out_chars))) return -1;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    // codes jump over a table far larger than the caches: the offset prefetched 16
    // rows ahead, the bytes 8 ahead (static schedule: a thread's rows are contiguous)
    if (i + 16 < n) __builtin_prefetch(&tab_off[codes[i + 16]]);
    if (i + 8 < n) __builtin_prefetch(tab_chars + tab_off[codes[i + 8]]);
    memcpy(out_chars + out_off[i], tab_chars + tab_off[codes[i]], (size_t)(out_off[i + 1] - out_off[i]));
  }
  return 0;
}

uint64_t qfio_hash_bytes(const void* data, int64_t nbytes) {
  if (!data || nbytes <= 0) return 0x9E3779B97F4A7C15ull ^ (uint64_t)(nbytes < 0 ? 0 : nbytes);
  // 1 MB blocks hashed in parallel (8-byte words, multiply-mix), then the block
  // hashes combined in order: a content digest for the pack cache (not a
  // cryptographic hash; any change of a word changes its block's value)
  const char* p = (const char*)data;
  constexpr int64_t kBlock = 1 << 20;
  const int64_t nb = (nbytes + kBlock - 1) / kBlock;
  std::vector<uint64_t> hb((size_t)nb);
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t a = b * kBlock, e = std::min(nbytes, a + kBlock);
    uint64_t h0 = 0x243F6A8885A308D3ull ^ (uint64_t)b, h1 = 0x13198A2E03707344ull;
    int64_t i = a;
    for (; i + 16 <= e; i += 16) {
      uint64_t w0, w1;
      memcpy(&w0, p + i, 8);
      memcpy(&w1, p + i + 8, 8);
      h0 = (h0 ^ w0) * 0xff51afd7ed558ccdull;
      h1 = (h1 ^ w1) * 0xc4ceb9fe1a85ec53ull;
      h0 ^= h0 >> 29;
      h1 ^= h1 >> 31;
    }
    // the tail (0-15 bytes): up to 8 into h0, the rest into h1
    if (i < e) {
      uint64_t w = 0;
      const int64_t n0 = std::min<int64_t>(8, e - i);
      memcpy(&w, p + i, (size_t)n0);
      h0 = (h0 ^ w ^ ((uint64_t)n0 << 56)) * 0xff51afd7ed558ccdull;
      i += n0;
    }
    if (i < e) {
      uint64_t w = 0;
      memcpy(&w, p + i, (size_t)(e - i));
      h1 = (h1 ^ w ^ ((uint64_t)(e - i) << 56)) * 0xc4ceb9fe1a85ec53ull;
    }
    hb[(size_t)b] = hash_words((const char*)&h0, 8) ^ (hash_words((const char*)&h1, 8) * 3);
  }
  return hash_words((const char*)hb.data(), hb.size() * 8) ^ (uint64_t)nbytes;
}

void qfio_repeat_offsets(int64_t len, int64_t n, int64_t* out_off) {
  if (n < 0 || !out_off) return;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i <= n; ++i) out_off[i] = i * len;
}

void qfio_runset_free(qfio_runset* rs) { delete rs; }

// ---- writer ---------------------------------------------------------------------

// Python's f"{x:.6f}".
static inline size_t fmt6(double x, char* out) {
  if (!(std::fabs(x) < 8589934592.0)) {  // 2^33, and inf / nan
    if (std::isnan(x)) {  // Python formats every NaN as "nan", whatever its sign bit
      memcpy(out, "nan", 3);
      return 3;
    }
    return (size_t)snprintf(out, 400, "%.6f", x);
  }
  // m = round-half-even(x * 1e6) on the exact binary value (as qf_common.h round6)
  double f = std::floor(x * 1e6);
  if (std::fma(x, 1e6, -f) < 0.0) f -= 1.0;
  else if (std::fma(x, 1e6, -(f + 1.0)) >= 0.0) f += 1.0;
  const double r = std::fma(x, 1e6, -(f + 0.5));
  long long m = (long long)f;
  if (r > 0.0 || (r == 0.0 && (m & 1))) m += 1;
  size_t n = 0;
  if (std::signbit(x)) out[n++] = '-';
  unsigned long long a = (unsigned long long)(m < 0 ? -m : m);
  const unsigned long long ip = a / 1000000ull, fp = a % 1000000ull;
  char tmp[24];
  int k = 0;
  unsigned long long v = ip;
  do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (k) out[n++] = tmp[--k];
  out[n++] = '.';
  char fd[6];
  unsigned long long w = fp;
  for (int i = 5; i >= 0; --i) { fd[i] = (char)('0' + w % 10); w /= 10; }
  memcpy(out + n, fd, 6);
  return n + 6;
}

size_t qfio_format_score(double x, char* out) { return fmt6(x, out); }

}  // extern "C"

// write_run's output file (see there): a temporary file renamed over a regular
// target, or the target itself opened in place.
struct AtomicTarget {
  std::string final_path, tmp_path;  // tmp_path empty: written in place
  bool seekable = true;
  static mode_t process_umask() {  // without umask()'s process-wide set-and-restore
    FILE* f = fopen("/proc/self/status", "r");
    unsigned m = 022;
    if (f) {
      char line[256];
      while (fgets(line, sizeof line, f))
        if (sscanf(line, "Umask: %o", &m) == 1) break;
      fclose(f);
    }
    return (mode_t)m;
  }
  int open_for(const char* path) {
    struct stat st;
    const bool exists = stat(path, &st) == 0;  // follows a symlink to its target
    if (!exists || S_ISREG(st.st_mode)) {
      char* rp = exists ? realpath(path, nullptr) : nullptr;
      final_path = rp ? rp : path;
      free(rp);
      const size_t slash = final_path.rfind('/');
      const std::string dir = slash == std::string::npos ? "." : final_path.substr(0, slash + 1);
      const std::string base = slash == std::string::npos ? final_path : final_path.substr(slash + 1);
      std::string tmpl = (slash == std::string::npos ? std::string() : dir) + "." + base +
                         ".qfio-XXXXXX";
      std::vector<char> buf(tmpl.begin(), tmpl.end());
      buf.push_back('\0');
      const int fd = mkstemp(buf.data());
      if (fd >= 0) {
        const mode_t mode = exists ? (st.st_mode & 07777) : (0666 & ~process_umask());
        if (fchmod(fd, mode) == 0) {
          tmp_path = buf.data();
          return fd;
        }
        close(fd);
        unlink(buf.data());
      }
    }
    // in place, as open(path, "w"): a device, a FIFO, or no room for a temporary
    final_path = path;
    tmp_path.clear();
    const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    if (fd >= 0) {
      struct stat fs;
      seekable = fstat(fd, &fs) == 0 && S_ISREG(fs.st_mode);
    }
    return fd;
  }
  void abandon() {
    if (!tmp_path.empty()) unlink(tmp_path.c_str());
  }
  bool commit() {
    if (tmp_path.empty()) return true;
    if (rename(tmp_path.c_str(), final_path.c_str()) == 0) return true;
    const int e = errno;
    unlink(tmp_path.c_str());
    errno = e;
    return false;
  }
};

// write_runfile for one fused run (include/qfio.h), either perm width
template <class Perm>
static int write_run(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                     const int32_t* counts, const uint32_t* union_docid, const Perm* perm,
                     const double* fused, const int64_t* qid_off, const char* qid_chars,
                     const int64_t* docno_off, const char* docno_chars, const char* tag,
                     int32_t n_threads) {
  if (!path || (n_out > 0 && (!order || !qbase || !counts || !union_docid || !perm || !fused ||
                              !qid_off || !qid_chars || !docno_off || !docno_chars || !tag)))
    return fail(QFIO_EINVAL, "qfio_write_run: bad arguments");
  if (n_threads > 0) omp_set_num_threads(n_threads);
  PhaseTimer tm;
  const size_t tl = strlen(tag);
  const int T = std::max(1, omp_get_max_threads());
  const int64_t chunks = std::min<int64_t>(std::max<int64_t>(n_out, 1), (int64_t)T * 8);
  // A regular (or absent) target in a writable directory is written to a temporary
  // file beside it (mkstemp in the directory of its real path, the existing file's
  // mode copied, else 0666 & ~umask as open(path, "w") gives) and renamed over it on
  // success, so a failure part way (out of memory, a short write) leaves an existing
  // run file as it was, as the reference's buffered write would until its first
  // flush; a symlink is written through (its target replaced).  Anything else —
  // /dev/null, a FIFO or /dev/stdout, a file in a directory we cannot create in — is
  // written in place like the reference's open(path, "w"), chunks strictly in order
  // (a pipe cannot seek).
  AtomicTarget tgt;
  const int fd = tgt.open_for(path);
  if (fd < 0) return fail(QFIO_EIO, std::string("cannot write ") + path + ": " + strerror(errno));
  const bool seq = !tgt.seekable;
  // Each chunk of queries is formatted into a raw buffer sized by an upper bound
  // (no per-field string appends, no snprintf for the rank) and written at its
  // offset as soon as the chunk before it has published its end: the writes (one
  // file's writes are serialised by the kernel) overlap the formatting of later
  // chunks instead of following all of it.  Chunks are handed out in increasing
  // order by an atomic ticket, so the chunk a thread waits on has already been
  // taken by a running thread (which waits only on earlier chunks): no deadlock,
  // whatever order an OpenMP schedule would have used.
  // (Measured, not kept: the file sized once, mapped, and every chunk copied in by
  // its own thread — 0.145-0.185 s per 390 MB run on the GPU box's host, the same
  // as format-all-then-pwrite: the page-cache copy is the bound either way.)
  std::vector<std::atomic<int64_t>> at((size_t)chunks + 1);
  for (auto& x : at) x.store(-1, std::memory_order_relaxed);
  at[0].store(0, std::memory_order_release);
  int err = 0, werr = 0;
  std::atomic<int64_t> ticket{0};
#pragma omp parallel reduction(| : err, werr)
  for (int64_t c = ticket.fetch_add(1, std::memory_order_relaxed); c < chunks;
       c = ticket.fetch_add(1, std::memory_order_relaxed)) {
    const int64_t a = n_out * c / chunks, b = n_out * (c + 1) / chunks;
    size_t cap = 1 << 16;
    for (int64_t i = a; i < b; ++i) {
      const int64_t q = order[i];
      if (counts[q] > 0)
        cap += (size_t)counts[q] * ((size_t)(qid_off[q + 1] - qid_off[q]) + tl + 48);
    }
    char* o = (char*)malloc(cap);
    size_t used = 0;
    for (int64_t i = a; i < b && o; ++i) {
      const int64_t q = order[i];
      const int64_t base = qbase[q];
      const int32_t n = counts[q];
      const char* qs = qid_chars + qid_off[q];
      const size_t ql = (size_t)(qid_off[q + 1] - qid_off[q]);
      for (int32_t k = 0; k < n; ++k) {
        // the docno table is far larger than the caches and a query's documents are
        // spread over it: its offset prefetched 16 lines ahead, its bytes 8 ahead
        if (k + 16 < n) __builtin_prefetch(&docno_off[union_docid[base + perm[base + k + 16]]]);
        if (k + 8 < n)
          __builtin_prefetch(docno_chars + docno_off[union_docid[base + perm[base + k + 8]]]);
        const int64_t u = base + perm[base + k];  // rank k's first-seen index
        const uint32_t d = union_docid[u];
        const size_t dl = (size_t)(docno_off[d + 1] - docno_off[d]);
        // a line is at most qid + docno + tag + 430 bytes (rank <= 10 digits, score < 400)
        if (cap - used < ql + dl + tl + 430) {
          cap = 2 * cap + ql + dl + tl + 430;
          char* g = (char*)realloc(o, cap);
          if (!g) { free(o); o = nullptr; break; }
          o = g;
        }
        char* w = o + used;
        memcpy(w, qs, ql);
        w += ql;
        memcpy(w, " Q0 ", 4);
        w += 4;
        memcpy(w, docno_chars + docno_off[d], dl);
        w += dl;
        *w++ = ' ';
        {  // rank k + 1, decimal
          char t[12];
          int m = 0;
          uint32_t v = (uint32_t)k + 1u;
          do { t[m++] = (char)('0' + v % 10u); v /= 10u; } while (v);
          while (m) *w++ = t[--m];
        }
        *w++ = ' ';
        w += fmt6(fused[u], w);
        *w++ = ' ';
        memcpy(w, tag, tl);
        w += tl;
        *w++ = '\n';
        used = (size_t)(w - o);
      }
    }
    if (!o) { err |= 1; used = 0; }
    // this chunk's offset: the previous chunk's end, published once it is formatted
    int64_t off;
    while ((off = at[(size_t)c].load(std::memory_order_acquire)) < 0) std::this_thread::yield();
    if (!seq) at[(size_t)c + 1].store(off + (int64_t)used, std::memory_order_release);
    size_t done = 0;
    while (o && done < used) {
      const ssize_t r = seq ? write(fd, o + done, used - done)
                            : pwrite(fd, o + done, used - done, (off_t)(off + (int64_t)done));
      if (r <= 0) { werr |= 1; break; }
      done += (size_t)r;
    }
    // in place on a stream: the next chunk writes only once this one is written
    if (seq) at[(size_t)c + 1].store(off + (int64_t)used, std::memory_order_release);
    free(o);
  }
  tm.mark("write: format + pwrite");
  const bool closed = close(fd) == 0;
  if (!closed || werr || err) {
    tgt.abandon();
    if (err) return fail(QFIO_EIO, "qfio_write_run: out of memory");
    return fail(QFIO_EIO, std::string("short write to ") + path);
  }
  if (!tgt.commit()) {
    const int e = errno;
    return fail(QFIO_EIO, std::string("cannot write ") + path + ": " + strerror(e));
  }
  tm.mark("write: close");
  return QFIO_OK;
}

extern "C" {

int qfio_write_run(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                   const int32_t* counts, const uint32_t* union_docid, const uint16_t* perm,
                   const double* fused, const int64_t* qid_off, const char* qid_chars,
                   const int64_t* docno_off, const char* docno_chars, const char* tag,
                   int32_t n_threads) {
  return write_run(path, n_out, order, qbase, counts, union_docid, perm, fused, qid_off, qid_chars,
                   docno_off, docno_chars, tag, n_threads);
}

int qfio_write_run32(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                     const int32_t* counts, const uint32_t* union_docid, const uint32_t* perm,
                     const double* fused, const int64_t* qid_off, const char* qid_chars,
                     const int64_t* docno_off, const char* docno_chars, const char* tag,
                     int32_t n_threads) {
  return write_run(path, n_out, order, qbase, counts, union_docid, perm, fused, qid_off, qid_chars,
                   docno_off, docno_chars, tag, n_threads);
}

}  // extern "C"

// ---- compute_qpp_for_res_file's read of a raw run (src/qpp.py:292-305) -------------
//
// Every line with >= 5 whitespace-separated fields adds float(field 5) to its qid's
// list, in file order, qids in first-appearance order (the reference's defaultdict);
// then each list is sorted descending — stable, so equal values (-0.0 and 0.0) keep
// file order, as Python's sorted(reverse=True) does — and sliced [:top_k].  Files
// whose Python reading this does not reproduce byte for byte (a byte >= 0x80 or in
// 0x1c-0x1f, which Python's str.split() may treat as whitespace; a lone '\r', a line
// break in text mode; digit-group underscores, which float() accepts; a NaN, which
// makes Python's sort order depend on its position) are reported as QFIO_EPYTHON:
// the caller reads those with the reference's own Python loop.
struct qfio_scorelists {
  std::vector<int64_t> qid_off;
  std::string qid_chars;
  std::vector<int64_t> list_off;
  std::vector<double> scores;
  int64_t n_rows = 0;
};

namespace {

inline bool ci_eq(std::string_view a, const char* b) {
  const size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i)
    if ((char)(a[i] | 0x20) != b[i]) return false;
  return true;
}

// Python's float(text) for one whitespace-free field: 0 = ok, 1 = not a float
// (ValueError), 2 = a form only Python's reader should judge (underscores).
int py_float(std::string_view t, double& v) {
  if (t.find('_') != std::string_view::npos) return 2;
  size_t i = 0;
  if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
  const std::string_view body = t.substr(i);
  if (ci_eq(body, "inf") || ci_eq(body, "infinity") || ci_eq(body, "nan")) {
    v = body[0] == 'n' || body[0] == 'N' ? NAN : INFINITY;
    if (t[0] == '-') v = -v;
    return 0;
  }
  size_t nd = 0;
  while (i < t.size() && t[i] >= '0' && t[i] <= '9') { ++i; ++nd; }
  if (i < t.size() && t[i] == '.') {
    ++i;
    while (i < t.size() && t[i] >= '0' && t[i] <= '9') { ++i; ++nd; }
  }
  if (nd == 0) return 1;
  if (i < t.size() && (t[i] == 'e' || t[i] == 'E')) {
    ++i;
    if (i < t.size() && (t[i] == '+' || t[i] == '-')) ++i;
    size_t ne = 0;
    while (i < t.size() && t[i] >= '0' && t[i] <= '9') { ++i; ++ne; }
    if (ne == 0) return 1;
  }
  if (i != t.size()) return 1;
  int32_t m = 0;
  bool mok = false;
  if (!parse_score(t, v, m, mok)) {  // long texts: strtod on a heap copy
    std::string s(t);
    v = strtod(s.c_str(), nullptr);
  }
  return 0;
}

}  // namespace

extern "C" {

int qfio_read_score_lists(const char* path, int32_t top_k, int32_t n_threads,
                          qfio_scorelists** out) {
  if (!path || !out) return fail(QFIO_EINVAL, "qfio_read_score_lists: bad arguments");
  *out = nullptr;
  if (n_threads > 0) omp_set_num_threads(n_threads);
  Mapped m;
  m.fd = open(path, O_RDONLY);
  if (m.fd < 0) return fail(QFIO_ENOENT, std::string("cannot open ") + path + ": " + strerror(errno));
  struct stat st;
  fstat(m.fd, &st);
  m.size = (size_t)st.st_size;
  if (m.size) {
    m.data = (const char*)mmap(nullptr, m.size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, m.fd, 0);
    if (m.data == MAP_FAILED) {
      m.data = nullptr;
      return fail(QFIO_EIO, std::string("cannot map ") + path);
    }
  }
  const int T = std::max(1, omp_get_max_threads());
  std::vector<const char*> cut((size_t)T + 1);
  cut[0] = m.data;
  cut[T] = m.data + m.size;
  for (int t = 1; t < T; ++t) {
    const char* x = m.data + (m.size * (size_t)t) / (size_t)T;
    while (x < cut[T] && x > m.data && x[-1] != '\n') ++x;
    cut[t] = std::max(x, cut[t - 1]);
  }
  // per chunk: rows (qid run index, score) and the qid runs (heads)
  struct Chunk {
    std::vector<std::string_view> head;  // qid of each run
    std::vector<uint32_t> run_len;
    std::vector<double> score;
    int code = 0;
    std::string err;
  };
  std::vector<Chunk> ch((size_t)T);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < T; ++t) {
    Chunk c;  // local, moved into ch[t] at the end: the Chunk headers share cache lines
    c.score.reserve((size_t)(cut[t + 1] - cut[t]) / 32 + 16);
    const char* p = cut[t];
    const char* end = cut[t + 1];
    while (p < end) {
      const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
      const char* e = nl ? nl : end;
      std::string_view f[5];
      int nf = 0;
      const char* q = p;
      for (const char* x = p; x < e; ++x) {  // the bytes Python would read otherwise
        const unsigned char b = (unsigned char)*x;
        if (b >= 0x80 || (b >= 0x1c && b <= 0x1f) || (b == '\r' && x + 1 != e)) {
          c.code = 2;
          break;
        }
      }
      if (c.code) break;
      while (nf < 5) {
        while (q < e && kSpace[(unsigned char)*q]) ++q;
        if (q >= e) break;
        const char* s = q;
        while (q < e && !kSpace[(unsigned char)*q]) ++q;
        f[nf++] = std::string_view(s, (size_t)(q - s));
      }
      p = nl ? nl + 1 : end;
      if (nf < 5) continue;  // src/qpp.py:295: lines with fewer fields are skipped
      double v;
      const int r = py_float(f[4], v);
      if (r == 1) {
        c.code = 1;
        c.err = "could not convert string to float: '" + std::string(f[4]) + "'";
        break;
      }
      if (r == 2 || v != v) {
        c.code = 2;
        break;
      }
      if (c.head.empty() || c.head.back() != f[0]) {
        c.head.push_back(f[0]);
        c.run_len.push_back(0);
      }
      ++c.run_len.back();
      c.score.push_back(v);
    }
    ch[(size_t)t] = std::move(c);
  }
  for (int t = 0; t < T; ++t) {  // the first failing chunk in file order decides
    if (ch[(size_t)t].code == 1) return fail(QFIO_EPARSE, ch[(size_t)t].err);
    if (ch[(size_t)t].code == 2) return fail(QFIO_EPYTHON, "needs the Python reader");
  }
  // qids in first-appearance order over the runs (few: one run per query and chunk)
  auto* res = new qfio_scorelists();
  std::vector<std::string_view> qids;
  std::vector<int64_t> qcount;
  struct SvHash {
    size_t operator()(std::string_view v) const { return (size_t)hash_sv(v); }
  };
  std::unordered_map<std::string_view, uint32_t, SvHash> idx;
  std::vector<std::vector<uint32_t>> run_q((size_t)T);
  for (int t = 0; t < T; ++t) {
    const Chunk& c = ch[(size_t)t];
    run_q[(size_t)t].resize(c.head.size());
    for (size_t k = 0; k < c.head.size(); ++k) {
      auto it = idx.find(c.head[k]);
      uint32_t id;
      if (it == idx.end()) {
        id = (uint32_t)qids.size();
        idx.emplace(c.head[k], id);
        qids.push_back(c.head[k]);
        qcount.push_back(0);
      } else {
        id = it->second;
      }
      run_q[(size_t)t][k] = id;
      qcount[id] += c.run_len[k];
    }
  }
  const int64_t Q = (int64_t)qids.size();
  // every query's scores in file order (runs placed in chunk order), then sorted
  std::vector<int64_t> full_off((size_t)Q + 1, 0);
  for (int64_t q = 0; q < Q; ++q) full_off[(size_t)q + 1] = full_off[(size_t)q] + qcount[(size_t)q];
  res->n_rows = full_off[(size_t)Q];
  std::vector<double> full((size_t)res->n_rows);
  {
    std::vector<int64_t> pos(full_off.begin(), full_off.end() - 1);
    std::vector<std::vector<int64_t>> dst((size_t)T);
    for (int t = 0; t < T; ++t) {
      const Chunk& c = ch[(size_t)t];
      dst[(size_t)t].resize(c.head.size());
      for (size_t k = 0; k < c.head.size(); ++k) {
        const uint32_t id = run_q[(size_t)t][k];
        dst[(size_t)t][k] = pos[id];
        pos[id] += c.run_len[k];
      }
    }
#pragma omp parallel for schedule(static, 1)
    for (int t = 0; t < T; ++t) {
      const Chunk& c = ch[(size_t)t];
      size_t a = 0;
      for (size_t k = 0; k < c.head.size(); ++k) {
        memcpy(&full[(size_t)dst[(size_t)t][k]], &c.score[a], c.run_len[k] * sizeof(double));
        a += c.run_len[k];
      }
    }
  }
  // sorted(scores, reverse=True)[:top_k]: Python's slice of a list of n
  auto keep = [&](int64_t n) -> int64_t {
    if (top_k >= 0) return std::min<int64_t>(n, top_k);
    return std::max<int64_t>(0, n + top_k);
  };
  res->list_off.assign((size_t)Q + 1, 0);
  for (int64_t q = 0; q < Q; ++q)
    res->list_off[(size_t)q + 1] = res->list_off[(size_t)q] + keep(qcount[(size_t)q]);
  res->scores.resize((size_t)res->list_off[(size_t)Q]);
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t q = 0; q < Q; ++q) {
    double* a = &full[(size_t)full_off[(size_t)q]];
    double* b = &full[(size_t)full_off[(size_t)q + 1]];
    std::stable_sort(a, b, [](double x, double y) { return x > y; });
    std::copy(a, a + keep(b - a), &res->scores[(size_t)res->list_off[(size_t)q]]);
  }
  res->qid_off.assign((size_t)Q + 1, 0);
  for (int64_t q = 0; q < Q; ++q)
    res->qid_off[(size_t)q + 1] = res->qid_off[(size_t)q] + (int64_t)qids[(size_t)q].size();
  res->qid_chars.reserve((size_t)res->qid_off[(size_t)Q]);
  for (const auto& v : qids) res->qid_chars.append(v.data(), v.size());
  *out = res;
  return QFIO_OK;
}

void qfio_scorelists_sizes(const qfio_scorelists* s, int64_t* sizes) {
  if (!s || !sizes) return;
  sizes[0] = (int64_t)s->list_off.size() - 1;
  sizes[1] = (int64_t)s->scores.size();
  sizes[2] = (int64_t)s->qid_chars.size();
  sizes[3] = s->n_rows;
}

int qfio_scorelists_get(const qfio_scorelists* s, int64_t* qid_off, char* qid_chars,
                        int64_t* list_off, double* scores) {
  if (!s || !qid_off || !list_off || (!qid_chars && !s->qid_chars.empty()) ||
      (!scores && !s->scores.empty()))
    return fail(QFIO_EINVAL, "qfio_scorelists_get: bad arguments");
  memcpy(qid_off, s->qid_off.data(), s->qid_off.size() * sizeof(int64_t));
  memcpy(list_off, s->list_off.data(), s->list_off.size() * sizeof(int64_t));
  if (!s->qid_chars.empty()) memcpy(qid_chars, s->qid_chars.data(), s->qid_chars.size());
  if (!s->scores.empty()) memcpy(scores, s->scores.data(), s->scores.size() * sizeof(double));
  return QFIO_OK;
}

void qfio_scorelists_free(qfio_scorelists* s) { delete s; }

}  // extern "C"
