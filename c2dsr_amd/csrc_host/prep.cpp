// Host-side data pipeline, C ABI declared in include/c2dsr_prep.h.
//
// Bit-exact with the reference's Python:
//   read_raw            dataloader.py:39-58, utils/graph.py:36-47   (items stable-sorted by timestamp)
//   preprocess_train    dataloader.py:60-161                         (14 index lists per sequence)
//   preprocess_evaluate dataloader.py:163-228                        (11 lists, random.sample negatives)
//   transition edges    utils/graph.py:54-81
// including the draws from CPython's global `random` (MT19937, Python 3.10 semantics):
//   randint(a, b)  = a + _randbelow(b - a + 1)
//   _randbelow(n)  = k = bit_length(n); r = getrandbits(k) until r < n;  getrandbits(k) = u32 >> (32 - k)
//   sample(pop, k) = pool path when len(pop) <= setsize (21 + 4**ceil(log(3k, 4)) for k > 5), else
//                    rejection against the selected set.
// The MT state is CPython's random.getstate()[1] (624 words + position), read and written back.
#include "../../include/c2dsr_prep.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// ---------------------------------------------------------------- MT19937 (CPython _randommodule.c)
struct MT {
  uint32_t s[624];
  int idx;

  void load(const uint32_t* st) {
    std::memcpy(s, st, sizeof(s));
    idx = (int)st[624];
  }
  void store(uint32_t* st) const {
    std::memcpy(st, s, sizeof(s));
    st[624] = (uint32_t)idx;
  }
  uint32_t next() {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    if (idx >= 624) {
      int kk;
      for (kk = 0; kk < 624 - 397; kk++) {
        y = (s[kk] & 0x80000000u) | (s[kk + 1] & 0x7fffffffu);
        s[kk] = s[kk + 397] ^ (y >> 1) ^ mag01[y & 1u];
      }
      for (; kk < 623; kk++) {
        y = (s[kk] & 0x80000000u) | (s[kk + 1] & 0x7fffffffu);
        s[kk] = s[kk + (397 - 624)] ^ (y >> 1) ^ mag01[y & 1u];
      }
      y = (s[623] & 0x80000000u) | (s[0] & 0x7fffffffu);
      s[623] = s[396] ^ (y >> 1) ^ mag01[y & 1u];
      idx = 0;
    }
    y = s[idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // random._randbelow_with_getrandbits (n < 2**32)
  int64_t below(int64_t n) {
    if (n <= 0) return 0;
    int k = 0;
    for (uint64_t v = (uint64_t)n; v; v >>= 1) ++k;
    for (;;) {
      const uint64_t r = next() >> (32 - k);
      if ((int64_t)r < n) return (int64_t)r;
    }
  }
  int64_t randint(int64_t a, int64_t b) { return a + below(b - a + 1); }
};

// ---------------------------------------------------------------- raw file
struct Seqs {
  std::vector<int64_t> off{0};
  std::vector<int64_t> items;
};

bool parse_i64(const char* b, const char* e, int64_t* out) {
  while (b < e && (*b == ' ' || *b == '\t' || *b == '\r' || *b == '\n')) ++b;
  while (e > b && (e[-1] == ' ' || e[-1] == '\t' || e[-1] == '\r' || e[-1] == '\n')) --e;
  if (b == e) return false;
  std::string s(b, e);
  char* end = nullptr;
  errno = 0;
  const long long v = std::strtoll(s.c_str(), &end, 10);
  if (errno || end != s.c_str() + s.size()) return false;
  *out = v;
  return true;
}

int read_file(const char* path, Seqs* S) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return fail(-2, std::string("cannot open ") + path);
  std::string buf;
  char chunk[1 << 16];
  size_t got;
  while ((got = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.append(chunk, got);
  std::fclose(f);
  std::vector<std::pair<int64_t, int64_t>> pairs;  // (ts, item)
  size_t pos = 0;
  int64_t lineno = 0;
  while (pos < buf.size()) {
    size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) nl = buf.size();
    ++lineno;
    // line.strip().split('\t')[2:]
    size_t b = pos, e = nl;
    while (b < e && std::isspace((unsigned char)buf[b])) ++b;
    while (e > b && std::isspace((unsigned char)buf[e - 1])) --e;
    pos = nl + 1;
    pairs.clear();
    int field = 0;
    size_t fb = b;
    for (size_t i = b; i <= e; ++i) {
      if (i == e || buf[i] == '\t') {
        if (field >= 2) {
          const char* p0 = buf.data() + fb;
          const char* p1 = buf.data() + i;
          const char* bar = (const char*)std::memchr(p0, '|', p1 - p0);
          if (!bar) return fail(-3, "line " + std::to_string(lineno) + ": field without item|timestamp");
          const char* bar2 = (const char*)std::memchr(bar + 1, '|', p1 - bar - 1);
          int64_t item, ts;
          if (!parse_i64(p0, bar, &item) || !parse_i64(bar + 1, bar2 ? bar2 : p1, &ts))
            return fail(-3, "line " + std::to_string(lineno) + ": bad item|timestamp");
          pairs.emplace_back(ts, item);
        }
        ++field;
        fb = i + 1;
      }
    }
    // list.sort(key=ts) is stable
    std::stable_sort(pairs.begin(), pairs.end(),
                     [](const std::pair<int64_t, int64_t>& x, const std::pair<int64_t, int64_t>& y) {
                       return x.first < y.first;
                     });
    for (auto& p : pairs) S->items.push_back(p.second);
    S->off.push_back((int64_t)S->items.size());
  }
  return 0;
}

// dataloader.py:97-133 — walk one domain view from the end
void targets_backwards(std::vector<int64_t>& seq, std::vector<int64_t>& pos, bool last_in_domain, int64_t last_local,
                       int64_t pad, int64_t offset, int64_t none, std::vector<int64_t>& gt, std::vector<int64_t>& mask) {
  const size_t n = seq.size();
  gt.assign(n, none);
  mask.assign(n, 0);
  int64_t cur = -1;
  bool have = false;
  for (size_t i = 1; i <= n; ++i) {
    const size_t k = n - i;
    if (!pos[k]) continue;
    if (!have) {
      have = true;
      cur = seq[k] - offset;
      if (last_in_domain) {
        gt[k] = last_local;
        mask[k] = 1;
      } else {
        seq[k] = pad;
        pos[k] = 0;
      }
    } else {
      gt[k] = cur;
      mask[k] = 1;
      cur = seq[k] - offset;
    }
  }
}

}  // namespace

extern "C" {

void* c2dsr_prep_open(const char* path) {
  auto* S = new Seqs();
  if (read_file(path, S) != 0) {
    delete S;
    return nullptr;
  }
  return S;
}

void c2dsr_prep_close(void* h) { delete (Seqs*)h; }

int c2dsr_prep_sizes(void* h, int64_t* n_seq, int64_t* n_items) {
  if (!h) return fail(-1, "null handle");
  const Seqs* S = (const Seqs*)h;
  *n_seq = (int64_t)S->off.size() - 1;
  *n_items = (int64_t)S->items.size();
  return 0;
}

int c2dsr_prep_sequences(void* h, int64_t* offsets, int64_t* items) {
  if (!h) return fail(-1, "null handle");
  const Seqs* S = (const Seqs*)h;
  std::memcpy(offsets, S->off.data(), S->off.size() * sizeof(int64_t));
  if (!S->items.empty()) std::memcpy(items, S->items.data(), S->items.size() * sizeof(int64_t));
  return 0;
}

int c2dsr_prep_train(void* h, int n_a, int n_b, int len_max, uint32_t* mt_state, int64_t* out, int64_t* n_out) {
  if (!h) return fail(-1, "null handle");
  const Seqs* S = (const Seqs*)h;
  MT mt;
  mt.load(mt_state);
  const int64_t pad = (int64_t)n_a + n_b;
  const int64_t L = len_max;
  int64_t rows = 0;
  std::vector<int64_t> seq, pos, sa, pa, na, sb, pb, nb, ga, ma, gb, mb;
  const int64_t n_seq = (int64_t)S->off.size() - 1;
  for (int64_t q = 0; q < n_seq; ++q) {
    const int64_t* u = S->items.data() + S->off[q];
    const int64_t n = S->off[q + 1] - S->off[q];
    if (n < 1) return fail(-4, "sequence " + std::to_string(q) + " is empty");
    const int64_t lp = L - n + 1;
    if (lp < 0) return fail(-5, "sequence " + std::to_string(q) + " is longer than len_max + 1");
    const int64_t last = u[n - 1];
    sa.clear(), pa.clear(), na.clear(), sb.clear(), pb.clear(), nb.clear();
    int64_t ca = 1, cb = 1;
    for (int64_t i = 0; i + 1 < n; ++i) {
      const int64_t idx = u[i];
      if (idx < n_a) {
        na.push_back(idx);
        sa.push_back(idx);
        pa.push_back(ca++);
        nb.push_back(mt.randint(0, n_a - 1));
        sb.push_back(pad);
        pb.push_back(0);
      } else {
        na.push_back(mt.randint(n_a, pad - 1));
        sa.push_back(pad);
        pa.push_back(0);
        nb.push_back(idx);
        sb.push_back(idx);
        pb.push_back(cb++);
      }
    }
    targets_backwards(sa, pa, last < n_a, last, pad, 0, n_a, ga, ma);
    bool any = false;
    for (int64_t v : ma) any |= v != 0;
    if (!any) continue;
    targets_backwards(sb, pb, last > n_a, last - n_a, pad, n_a, n_b, gb, mb);  // '>' as the reference (Q13)
    any = false;
    for (int64_t v : mb) any |= v != 0;
    if (!any) continue;
    int64_t* o = out + rows * 14 * L;
    auto put = [&](int f, int64_t padv, const int64_t* x) {
      int64_t* r = o + f * L;
      for (int64_t i = 0; i < lp; ++i) r[i] = padv;
      for (int64_t i = 0; i + 1 < n; ++i) r[lp + i] = x[i];
    };
    put(0, pad, u);
    put(1, pad, sa.data());
    put(2, pad, sb.data());
    for (int64_t i = 0; i < L; ++i) o[3 * L + i] = i < lp ? 0 : i - lp + 1;
    put(4, 0, pa.data());
    put(5, 0, pb.data());
    // gt = u[1:], padded with pad; share targets mapped per domain
    for (int64_t i = 0; i < L; ++i) {
      const int64_t g = i < lp ? pad : u[i - lp + 1];
      o[6 * L + i] = g < n_a ? g : n_a;
      o[7 * L + i] = g >= n_a ? g - n_a : n_b;
    }
    put(8, n_a, ga.data());
    put(9, n_b, gb.data());
    put(10, 0, ma.data());
    put(11, 0, mb.data());
    put(12, pad, na.data());
    put(13, pad, nb.data());
    ++rows;
  }
  *n_out = rows;
  mt.store(mt_state);
  return 0;
}

int c2dsr_prep_eval(void* h, int n_a, int n_b, int len_max, int n_neg, uint32_t* mt_state, int64_t* seqs,
                    int64_t* last, int64_t* neg) {
  if (!h) return fail(-1, "null handle");
  const Seqs* S = (const Seqs*)h;
  MT mt;
  mt.load(mt_state);
  const int64_t pad = (int64_t)n_a + n_b;
  const int64_t L = len_max;
  const int64_t n_seq = (int64_t)S->off.size() - 1;
  std::vector<int64_t> pool;
  std::unordered_set<int64_t> selected;
  int64_t setsize = 21;
  if (n_neg > 5) setsize += (int64_t)std::llround(std::pow(4.0, std::ceil(std::log((double)n_neg * 3) / std::log(4.0))));
  for (int64_t q = 0; q < n_seq; ++q) {
    const int64_t* u = S->items.data() + S->off[q];
    const int64_t n = S->off[q + 1] - S->off[q];
    if (n < 1) return fail(-4, "sequence " + std::to_string(q) + " is empty");
    const int64_t lp = L - n + 1;
    if (lp < 0) return fail(-5, "sequence " + std::to_string(q) + " is longer than len_max + 1");
    int64_t* o = seqs + q * 6 * L;
    for (int f = 0; f < 6; ++f)
      for (int64_t i = 0; i < lp; ++i) o[f * L + i] = f < 3 ? pad : 0;
    int64_t ca = 1, cb = 1;
    for (int64_t i = 0; i + 1 < n; ++i) {
      const int64_t idx = u[i], j = lp + i;
      o[0 * L + j] = idx;
      o[3 * L + j] = i + 1;
      if (idx < n_a) {
        o[1 * L + j] = idx, o[4 * L + j] = ca++;
        o[2 * L + j] = pad, o[5 * L + j] = 0;
      } else {
        o[1 * L + j] = pad, o[4 * L + j] = 0;
        o[2 * L + j] = idx, o[5 * L + j] = cb++;
      }
    }
    auto last_idx = [&](const int64_t* p) -> int64_t {
      for (int64_t i = 1; i <= L; ++i)
        if (p[L - i]) return L - i;
      return -1;
    };
    const int64_t g = u[n - 1];
    int64_t* l4 = last + q * 4;
    l4[0] = last_idx(o + 4 * L);
    l4[1] = last_idx(o + 5 * L);
    // population = range(t) + range(t + 1, hi), element j -> j < t ? j : j + 1
    int64_t t, hi;
    if (g < n_a) {
      l4[2] = 0, l4[3] = g, t = g, hi = n_a;
    } else {
      l4[2] = 1, l4[3] = g - n_a, t = g - n_a, hi = (int64_t)n_b - n_a;  // Q14: range(n_b - n_a)
    }
    const int64_t npop = std::max<int64_t>(t, 0) + std::max<int64_t>(hi - (t + 1), 0);
    const int64_t t_eff = std::min<int64_t>(std::max<int64_t>(t, 0), npop);
    auto elem = [&](int64_t j) { return j < t_eff ? j : (t + 1) + (j - t_eff); };
    if (n_neg > npop) return fail(-6, "sequence " + std::to_string(q) + ": sample larger than population");
    int64_t* r = neg + q * n_neg;
    if (npop <= setsize) {
      pool.resize(npop);
      for (int64_t j = 0; j < npop; ++j) pool[j] = elem(j);
      for (int64_t i = 0; i < n_neg; ++i) {
        const int64_t j = mt.below(npop - i);
        r[i] = pool[j];
        pool[j] = pool[npop - i - 1];
      }
    } else {
      selected.clear();
      for (int64_t i = 0; i < n_neg; ++i) {
        int64_t j = mt.below(npop);
        while (selected.count(j)) j = mt.below(npop);
        selected.insert(j);
        r[i] = elem(j);
      }
    }
  }
  mt.store(mt_state);
  return 0;
}

int c2dsr_prep_edges(void* h, int n_a, int64_t* share, int64_t* n_share, int64_t* spec, int64_t* n_spec) {
  if (!h) return fail(-1, "null handle");
  const Seqs* S = (const Seqs*)h;
  int64_t ns = 0, np = 0;
  const int64_t n_seq = (int64_t)S->off.size() - 1;
  for (int64_t q = 0; q < n_seq; ++q) {
    int64_t src = -1, tgt = -1, pre = -1;
    for (int64_t i = S->off[q]; i < S->off[q + 1]; ++i) {
      const int64_t d = S->items[i];
      if (d < n_a) {
        if (src != -1) spec[2 * np] = src, spec[2 * np + 1] = d, ++np;
        src = d;
      } else {
        if (tgt != -1) spec[2 * np] = tgt, spec[2 * np + 1] = d, ++np;
        tgt = d;
      }
      if (pre != -1) share[2 * ns] = pre, share[2 * ns + 1] = d, ++ns;
      pre = d;
    }
  }
  *n_share = ns;
  *n_spec = np;
  return 0;
}

const char* c2dsr_prep_error(void) { return g_err.c_str(); }

}  // extern "C"
