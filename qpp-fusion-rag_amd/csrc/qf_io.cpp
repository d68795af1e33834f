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
#include <fcntl.h>
#include <omp.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <parallel/algorithm>
#include <string>
#include <string_view>
#include <vector>

#include "../../include/qfio.h"

namespace {

thread_local std::string g_err;

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

struct Row {
  std::string_view qid, iter, docno, tag;
  int64_t rank;
  double score;
  int32_t micro;
  bool micro_ok;
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

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

// Parse [begin, end) of a mapped file (whole lines) into rows.
bool parse_chunk(const char* p, const char* end, std::vector<Row>& rows, std::string& err) {
  while (p < end) {
    std::string_view f[7];
    int nf = 0;
    const char* line = p;
    while (p < end && *p != '\n') {
      while (p < end && is_space(*p)) ++p;
      if (p >= end || *p == '\n') break;
      const char* s = p;
      while (p < end && *p != '\n' && !is_space(*p)) ++p;
      if (nf < 7) f[nf] = std::string_view(s, (size_t)(p - s));
      ++nf;
    }
    if (p < end) ++p;  // '\n'
    if (nf == 0) continue;  // blank line (pandas skips it)
    if (nf != 6) {
      err = "expected 6 fields (qid Q0 docno rank score tag), got " + std::to_string(nf) +
            " in line: " + std::string(line, std::min<size_t>(120, (size_t)(p - line)));
      return false;
    }
    Row r;
    r.qid = f[0];
    r.iter = f[1];
    r.docno = f[2];
    r.tag = f[5];
    char buf[32];
    if (f[3].size() >= sizeof buf) { err = "bad rank field"; return false; }
    memcpy(buf, f[3].data(), f[3].size());
    buf[f[3].size()] = 0;
    char* e2 = nullptr;
    r.rank = strtoll(buf, &e2, 10);
    if (e2 != buf + f[3].size()) { err = "bad rank field '" + std::string(f[3]) + "'"; return false; }
    r.micro = 0;
    if (!parse_score(f[4], r.score, r.micro, r.micro_ok)) {
      err = "bad score field '" + std::string(f[4]) + "'";
      return false;
    }
    rows.push_back(r);
  }
  return true;
}

inline uint64_t hash_sv(std::string_view v) {  // FNV-1a + avalanche
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : v) h = (h ^ c) * 1099511628211ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h;
}

// Sorted unique strings of `views`, and each view's index among them: hash
// partitions deduplicated in parallel, then only the distinct strings sorted.
void intern(const std::vector<std::string_view>& views, std::vector<std::string_view>& uniq,
            std::vector<uint32_t>& id) {
  const size_t n = views.size();
  constexpr int P = 256;
  std::vector<uint64_t> hs(n);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) hs[i] = hash_sv(views[i]);
  // rows of each partition (top 8 bits), in row order
  const int T = std::max(1, omp_get_max_threads());
  std::vector<std::vector<uint32_t>> cnt(T, std::vector<uint32_t>(P, 0));
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T; ++t)
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) ++cnt[t][hs[i] >> 56];
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
  std::vector<uint32_t> rows(n);
#pragma omp parallel for schedule(static)
  for (int t = 0; t < T; ++t)
    for (size_t i = n * t / T; i < n * (t + 1) / T; ++i) rows[at[t][hs[i] >> 56]++] = (uint32_t)i;
  // per partition: open-addressing table of first rows -> local unique index
  std::vector<std::vector<uint32_t>> ufirst(P);  // first row of each distinct string
  std::vector<uint32_t> local(n);
#pragma omp parallel for schedule(dynamic, 4)
  for (int b = 0; b < P; ++b) {
    const size_t a0 = start[b], a1 = start[b + 1], m = a1 - a0;
    if (!m) continue;
    size_t cap = 16;
    while (cap < 2 * m) cap <<= 1;
    std::vector<uint32_t> tab(cap, 0xFFFFFFFFu);
    auto& uf = ufirst[b];
    for (size_t k = a0; k < a1; ++k) {
      const uint32_t i = rows[k];
      size_t h = (size_t)hs[i] & (cap - 1);
      while (true) {
        const uint32_t u = tab[h];
        if (u == 0xFFFFFFFFu) {
          tab[h] = (uint32_t)uf.size();
          local[i] = (uint32_t)uf.size();
          uf.push_back(i);
          break;
        }
        const uint32_t r = uf[u];
        if (hs[r] == hs[i] && views[r] == views[i]) { local[i] = u; break; }
        h = (h + 1) & (cap - 1);
      }
    }
  }
  std::vector<size_t> ubase(P + 1, 0);
  for (int b = 0; b < P; ++b) ubase[b + 1] = ubase[b] + ufirst[b].size();
  const size_t U = ubase[P];
  std::vector<uint32_t> reps(U);  // row of each distinct string
  for (int b = 0; b < P; ++b)
    std::copy(ufirst[b].begin(), ufirst[b].end(), reps.begin() + (long)ubase[b]);
  std::vector<uint32_t> order(U);
  for (size_t k = 0; k < U; ++k) order[k] = (uint32_t)k;
  __gnu_parallel::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    return views[reps[a]] < views[reps[b]];  // byte order == Python's str order for UTF-8
  });
  std::vector<uint32_t> rank(U);
  uniq.resize(U);
  for (size_t k = 0; k < U; ++k) {
    rank[order[k]] = (uint32_t)k;
    uniq[k] = views[reps[order[k]]];
  }
  id.resize(n);
#pragma omp parallel for schedule(static)
  for (size_t i = 0; i < n; ++i) id[i] = rank[ubase[hs[i] >> 56] + local[i]];
}

}  // namespace

struct qfio_runset {
  std::vector<Mapped*> maps;
  int32_t n_files = 0;
  std::vector<std::string_view> qids, docnos, iters, tags;
  // CSR (query-major, run-minor), rows in file order
  std::vector<int64_t> list_off;
  std::vector<uint32_t> docid;
  std::vector<double> score;
  std::vector<int32_t> micro;
  std::vector<int64_t> rank;
  bool micro_ok = true;
  // per-file rows in file order (for DataFrames): codes and values
  std::vector<int64_t> file_off;  // [n_files + 1]
  std::vector<uint32_t> row_qid, row_docid, row_iter, row_tag;
  std::vector<int64_t> row_rank;
  std::vector<double> row_score;
  ~qfio_runset() {
    for (auto* m : maps) delete m;
  }
};

extern "C" {

const char* qfio_last_error(void) { return g_err.c_str(); }

int qfio_load_runs(const char* const* paths, int32_t n_files, int32_t n_threads,
                   qfio_runset** out) {
  if (!paths || n_files <= 0 || !out) return fail(QFIO_EINVAL, "qfio_load_runs: bad arguments");
  if (n_threads > 0) omp_set_num_threads(n_threads);
  auto* rs = new qfio_runset();
  rs->n_files = n_files;
  std::vector<std::vector<Row>> per_file(n_files);
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
      m->data = (const char*)mmap(nullptr, m->size, PROT_READ, MAP_PRIVATE, m->fd, 0);
      if (m->data == MAP_FAILED) {
        m->data = nullptr;
        delete rs;
        return fail(QFIO_EIO, std::string("cannot map ") + paths[f]);
      }
      madvise((void*)m->data, m->size, MADV_SEQUENTIAL);
    }
    // chunk at line boundaries
    const int T = std::max(1, omp_get_max_threads());
    std::vector<const char*> cut(T + 1);
    cut[0] = m->data;
    cut[T] = m->data + m->size;
    for (int t = 1; t < T; ++t) {
      const char* c = m->data + (m->size * (size_t)t) / (size_t)T;
      while (c < cut[T] && c > m->data && c[-1] != '\n') ++c;
      cut[t] = std::max(c, cut[t - 1]);
    }
    std::vector<std::vector<Row>> parts(T);
    std::vector<std::string> errs(T);
    int bad = 0;
#pragma omp parallel for schedule(static, 1) reduction(+ : bad)
    for (int t = 0; t < T; ++t) {
      parts[t].reserve((size_t)(cut[t + 1] - cut[t]) / 40 + 16);
      if (!parse_chunk(cut[t], cut[t + 1], parts[t], errs[t])) bad += 1;
    }
    for (int t = 0; t < T; ++t)
      if (!errs[t].empty()) {
        const std::string e = std::string(paths[f]) + ": " + errs[t];
        delete rs;
        return fail(QFIO_EPARSE, e);
      }
    size_t n = 0;
    for (auto& v : parts) n += v.size();
    per_file[f].reserve(n);
    for (auto& v : parts) per_file[f].insert(per_file[f].end(), v.begin(), v.end());
  }
  // ---- flatten (file order), intern qids / docnos / iter / tag -----------------
  rs->file_off.assign(n_files + 1, 0);
  for (int f = 0; f < n_files; ++f) rs->file_off[f + 1] = rs->file_off[f] + (int64_t)per_file[f].size();
  const size_t E = (size_t)rs->file_off[n_files];
  if (E >= 0xFFFFFFFFull) { delete rs; return fail(QFIO_EINVAL, "too many rows"); }
  std::vector<std::string_view> vq(E), vd(E), vi(E), vt(E);
  rs->row_rank.resize(E);
  rs->row_score.resize(E);
  std::vector<int32_t> row_micro(E);
  int micro_bad = 0;
  for (int f = 0; f < n_files; ++f) {
    const int64_t o = rs->file_off[f];
    const auto& rows = per_file[f];
#pragma omp parallel for schedule(static) reduction(+ : micro_bad)
    for (int64_t i = 0; i < (int64_t)rows.size(); ++i) {
      const Row& r = rows[i];
      vq[o + i] = r.qid;
      vd[o + i] = r.docno;
      vi[o + i] = r.iter;
      vt[o + i] = r.tag;
      rs->row_rank[o + i] = r.rank;
      rs->row_score[o + i] = r.score;
      row_micro[o + i] = r.micro;
      micro_bad += !r.micro_ok;
    }
    std::vector<Row>().swap(per_file[f]);
  }
  rs->micro_ok = micro_bad == 0;
  intern(vq, rs->qids, rs->row_qid);
  intern(vd, rs->docnos, rs->row_docid);
  intern(vi, rs->iters, rs->row_iter);
  intern(vt, rs->tags, rs->row_tag);
  if (rs->docnos.size() >= 0xFFFFFFFFull) { delete rs; return fail(QFIO_EINVAL, "too many docnos"); }
  // ---- CSR by (query, file), stable in file order -------------------------------
  const int64_t Q = (int64_t)rs->qids.size(), R = n_files;
  std::vector<int64_t> cnt(Q * R + 1, 0);
  for (int f = 0; f < n_files; ++f)
    for (int64_t i = rs->file_off[f]; i < rs->file_off[f + 1]; ++i) ++cnt[(int64_t)rs->row_qid[i] * R + f];
  rs->list_off.assign(Q * R + 1, 0);
  for (int64_t k = 0; k < Q * R; ++k) rs->list_off[k + 1] = rs->list_off[k] + cnt[k];
  std::vector<int64_t> pos(rs->list_off.begin(), rs->list_off.end() - 1);
  rs->docid.resize(E);
  rs->score.resize(E);
  rs->rank.resize(E);
  rs->micro.resize(rs->micro_ok ? E : 0);
  for (int f = 0; f < n_files; ++f)
    for (int64_t i = rs->file_off[f]; i < rs->file_off[f + 1]; ++i) {
      const int64_t d = pos[(int64_t)rs->row_qid[i] * R + f]++;
      rs->docid[d] = rs->row_docid[i];
      rs->score[d] = rs->row_score[i];
      rs->rank[d] = rs->row_rank[i];
      if (rs->micro_ok) rs->micro[d] = row_micro[i];
    }
  *out = rs;
  return QFIO_OK;
}

void qfio_runset_sizes(const qfio_runset* rs, int64_t* sizes /* [8] */) {
  int64_t qb = 0, db = 0, ib = 0, tb = 0;
  for (auto& s : rs->qids) qb += (int64_t)s.size();
  for (auto& s : rs->docnos) db += (int64_t)s.size();
  for (auto& s : rs->iters) ib += (int64_t)s.size();
  for (auto& s : rs->tags) tb += (int64_t)s.size();
  sizes[0] = (int64_t)rs->qids.size();
  sizes[1] = (int64_t)rs->docnos.size();
  sizes[2] = (int64_t)rs->docid.size();
  sizes[3] = qb;
  sizes[4] = db;
  sizes[5] = rs->micro_ok ? 1 : 0;
  sizes[6] = (int64_t)rs->iters.size() | ((int64_t)rs->tags.size() << 32);
  sizes[7] = ib | (tb << 32);
}

static void copy_strings(const std::vector<std::string_view>& v, int64_t* off, char* chars) {
  int64_t o = 0;
  off[0] = 0;
  for (size_t i = 0; i < v.size(); ++i) {
    memcpy(chars + o, v[i].data(), v[i].size());
    o += (int64_t)v[i].size();
    off[i + 1] = o;
  }
}

int qfio_runset_csr(const qfio_runset* rs, int64_t* list_off, uint32_t* docid, double* score,
                    int32_t* micro, int64_t* rank) {
  memcpy(list_off, rs->list_off.data(), rs->list_off.size() * sizeof(int64_t));
  memcpy(docid, rs->docid.data(), rs->docid.size() * sizeof(uint32_t));
  memcpy(score, rs->score.data(), rs->score.size() * sizeof(double));
  memcpy(rank, rs->rank.data(), rs->rank.size() * sizeof(int64_t));
  if (micro && rs->micro_ok) memcpy(micro, rs->micro.data(), rs->micro.size() * sizeof(int32_t));
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

int qfio_runset_rows(const qfio_runset* rs, int64_t* file_off, uint32_t* qid, uint32_t* docid,
                     uint32_t* iter, uint32_t* tag, int64_t* rank, double* score) {
  const size_t E = rs->row_qid.size();
  memcpy(file_off, rs->file_off.data(), rs->file_off.size() * sizeof(int64_t));
  memcpy(qid, rs->row_qid.data(), E * sizeof(uint32_t));
  memcpy(docid, rs->row_docid.data(), E * sizeof(uint32_t));
  memcpy(iter, rs->row_iter.data(), E * sizeof(uint32_t));
  memcpy(tag, rs->row_tag.data(), E * sizeof(uint32_t));
  memcpy(rank, rs->row_rank.data(), E * sizeof(int64_t));
  memcpy(score, rs->row_score.data(), E * sizeof(double));
  return QFIO_OK;
}

void qfio_runset_free(qfio_runset* rs) { delete rs; }

// ---- writer ---------------------------------------------------------------------

// Python's f"{x:.6f}".
static inline size_t fmt6(double x, char* out) {
  if (!(std::fabs(x) < 8589934592.0)) {  // 2^33, and inf / nan
    if (std::isnan(x)) return (size_t)snprintf(out, 48, "%snan", std::signbit(x) ? "-" : "");
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

int qfio_write_run(const char* path, int64_t n_out, const int64_t* order, const int64_t* qbase,
                   const int32_t* counts, const uint32_t* union_docid, const uint16_t* perm,
                   const double* fused, const int64_t* qid_off, const char* qid_chars,
                   const int64_t* docno_off, const char* docno_chars, const char* tag,
                   int32_t n_threads) {
  if (!path || (n_out > 0 && (!order || !qbase || !counts || !union_docid || !perm || !fused ||
                              !qid_off || !qid_chars || !docno_off || !docno_chars || !tag)))
    return fail(QFIO_EINVAL, "qfio_write_run: bad arguments");
  if (n_threads > 0) omp_set_num_threads(n_threads);
  const size_t tl = strlen(tag);
  const int T = std::max(1, omp_get_max_threads());
  const int64_t chunks = std::min<int64_t>(std::max<int64_t>(n_out, 1), (int64_t)T * 8);
  std::vector<std::string> buf((size_t)chunks);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t c = 0; c < chunks; ++c) {
    const int64_t a = n_out * c / chunks, b = n_out * (c + 1) / chunks;
    std::string& s = buf[(size_t)c];
    size_t est = 0;
    for (int64_t i = a; i < b; ++i) est += (size_t)std::max(counts[order[i]], 0) * (48 + tl);
    s.reserve(est);
    char line[512];
    for (int64_t i = a; i < b; ++i) {
      const int64_t q = order[i];
      const int64_t base = qbase[q];
      const int32_t n = counts[q];
      const std::string_view qid(qid_chars + qid_off[q], (size_t)(qid_off[q + 1] - qid_off[q]));
      for (int32_t k = 0; k < n; ++k) {
        const uint32_t d = union_docid[base + perm[base + k]];
        size_t o = 0;
        memcpy(line + o, qid.data(), qid.size());
        o += qid.size();
        memcpy(line + o, " Q0 ", 4);
        o += 4;
        s.append(line, o);
        s.append(docno_chars + docno_off[d], (size_t)(docno_off[d + 1] - docno_off[d]));
        o = 0;
        line[o++] = ' ';
        o += (size_t)snprintf(line + o, 32, "%d", k + 1);
        line[o++] = ' ';
        o += fmt6(fused[base + k], line + o);
        line[o++] = ' ';
        s.append(line, o);
        s.append(tag, tl);
        s.push_back('\n');
      }
    }
  }
  FILE* fp = fopen(path, "wb");
  if (!fp) return fail(QFIO_EIO, std::string("cannot write ") + path + ": " + strerror(errno));
  for (auto& s : buf)
    if (!s.empty() && fwrite(s.data(), 1, s.size(), fp) != s.size()) {
      fclose(fp);
      return fail(QFIO_EIO, std::string("short write to ") + path);
    }
  if (fclose(fp) != 0) return fail(QFIO_EIO, std::string("cannot close ") + path);
  return QFIO_OK;
}

}  // extern "C"
