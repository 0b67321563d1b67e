// kfserve_host.cpp — libkfserve.so: native v1 request-body parser
// (include/kfserve.h).  Host code only; no GPU.
//
// Replaces, for the common body shape, the json.loads + list -> ndarray
// conversion of the reference serving path (handlers/http.py:69,
// xgbserver/model.py:46, sklearnserver/model.py:46).  Exactness: a number
// with a decimal significand w < 2^53 and a power of ten 10^e, |e| <= 22, is
// one correctly rounded IEEE operation w * 10^e or w / 10^-e (Clinger's fast
// path); every other number goes to strtod, which is correctly rounded in
// glibc -- the same result as Python's float(text); significands of at most
// 19 digits take the Eisel-Lemire conversion instead (exact, ~10x faster).  Integer literals of up
// to 18 digits convert exactly as Python's int -> float (round to nearest
// even), which is what numpy does with them.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kfserve.h"
#include "pow5_table.h"

namespace {

// Eisel-Lemire (Lemire 2021, as in the fast_float library): the correctly
// rounded binary64 nearest to w * 10^q for a nonzero decimal significand w
// of at most 19 digits, q in [-342, 308], from one or two 64x128-bit
// products with the truncated power of five.  Mushtak & Lemire (2023) show
// the result needs no fallback for such w.
double eisel_lemire(uint64_t w, int64_t q, bool neg) {
  const uint64_t sign = neg ? (uint64_t(1) << 63) : 0;
  auto bits = [&](uint64_t m, int64_t p2) {
    const uint64_t b = sign | (static_cast<uint64_t>(p2) << 52) | m;
    double d;
    std::memcpy(&d, &b, 8);
    return d;
  };
  if (w == 0 || q < -342) return bits(0, 0);
  if (q > 308) return bits(0, 0x7FF);
  const int lz = __builtin_clzll(w);
  w <<= lz;
  const int idx = 2 * static_cast<int>(q + 342);
  unsigned __int128 first = static_cast<unsigned __int128>(w) * kPow5_128[idx];
  uint64_t hi = static_cast<uint64_t>(first >> 64), lo = static_cast<uint64_t>(first);
  const uint64_t mask = 0xFFFFFFFFFFFFFFFFULL >> 55;   // 52 + 3 bits of precision
  if ((hi & mask) == mask) {
    const unsigned __int128 second = static_cast<unsigned __int128>(w) * kPow5_128[idx + 1];
    const uint64_t shi = static_cast<uint64_t>(second >> 64);
    lo += shi;
    if (shi > lo) ++hi;
  }
  const int upper = static_cast<int>(hi >> 63);
  const int shift = upper + 64 - 52 - 3;
  uint64_t m = hi >> shift;
  int64_t p2 = ((((152170 + 65536) * q) >> 16) + 63) + upper - lz + 1023;
  if (p2 <= 0) {   // subnormal
    if (-p2 + 1 >= 64) return bits(0, 0);
    m >>= -p2 + 1;
    m += (m & 1);
    m >>= 1;
    p2 = m < (uint64_t(1) << 52) ? 0 : 1;
    return bits(m & ~(uint64_t(1) << 52), p2);
  }
  if (lo <= 1 && q >= -4 && q <= 23 && (m & 3) == 1 && (m << shift) == hi) m &= ~uint64_t(1);
  m += (m & 1);
  m >>= 1;
  if (m >= (uint64_t(2) << 52)) {
    m = uint64_t(1) << 52;
    ++p2;
  }
  m &= ~(uint64_t(1) << 52);
  if (p2 >= 0x7FF) return bits(0, 0x7FF);
  return bits(m, p2);
}

const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

struct Scanner {
  const char* p;
  const char* end;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool eat(char c) {
    if (p < end && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
  bool lit(const char* s, size_t n) {
    if (static_cast<size_t>(end - p) >= n && std::memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static bool digit(char c) { return c >= '0' && c <= '9'; }

  static uint64_t load8(const char* q) {
    uint64_t v;
    std::memcpy(&v, q, 8);
    return v;
  }
  // Number of leading ASCII digits in the 8 bytes of v (0..8).
  static int digit_run(uint64_t v) {
    const uint64_t x = v ^ 0x3030303030303030ULL;   // digits -> 0..9
    const uint64_t bad = ((x + 0x7676767676767676ULL) | x) & 0x8080808080808080ULL;
    return bad ? (__builtin_ctzll(bad) >> 3) : 8;
  }
  static uint32_t parse_eight(uint64_t v) {   // SWAR: 8 ASCII digits -> value
    v = (v & 0x0F0F0F0F0F0F0F0FULL) * 2561 >> 8;
    v = (v & 0x00FF00FF00FF00FFULL) * 6553601 >> 16;
    return static_cast<uint32_t>((v & 0x0000FFFF0000FFFFULL) * 42949672960001ULL >> 32);
  }
  // The first n (1..7) digits of v as a number: shift them to the top and
  // pad the low bytes with '0' (little endian: byte 0 is the first char).
  static uint32_t parse_head(uint64_t v, int n) {
    const int sh = (8 - n) * 8;
    return parse_eight((v << sh) | (0x3030303030303030ULL >> (64 - sh)));
  }

  static constexpr uint64_t kP10[9] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000,
                                       100000000};

  // Scan a run of digits at p into w.  Returns the run length; sets *ok =
  // false if the run would push w past 19 digits (nd counts digits in w).
  size_t digits(uint64_t& w, int& nd, bool* ok) {
    const char* q = p;
    if (end - p >= 16) {   // fast path: whole words readable
      for (;;) {
        const uint64_t v = load8(p);
        const int n = digit_run(v);
        if (n == 0) break;
        if (nd + n > 19) {
          *ok = false;
          while (p < end && digit(*p)) ++p;
          return static_cast<size_t>(p - q);
        }
        w = w * kP10[n] + (n == 8 ? parse_eight(v) : parse_head(v, n));
        nd += n;
        p += n;
        if (n < 8 || end - p < 8) break;
      }
    }
    while (p < end && digit(*p)) {
      if (nd >= 19) {
        *ok = false;
        while (p < end && digit(*p)) ++p;
        break;
      }
      w = w * 10 + static_cast<uint64_t>(*p - '0');
      ++nd;
      ++p;
    }
    return static_cast<size_t>(p - q);
  }

  // One JSON number (Python json's NUMBER_RE) or NaN / Infinity / -Infinity.
  bool number(double* v) {
    const char* s = p;
    if (p >= end) return false;
    const char c0 = *p;
    if (c0 == 'N') {
      if (!lit("NaN", 3)) return false;
      *v = std::nan("");
      return true;
    }
    if (c0 == 'I') {
      if (!lit("Infinity", 8)) return false;
      *v = HUGE_VAL;
      return true;
    }
    bool neg = false;
    if (c0 == '-') {
      if (end - p > 1 && p[1] == 'I') {
        if (!lit("-Infinity", 9)) return false;
        *v = -HUGE_VAL;
        return true;
      }
      neg = true;
      ++p;
    }
    if (p >= end || !digit(*p)) return false;
    uint64_t w = 0;
    int nd = 0;
    bool fits = true;                   // every significant digit is in w
    size_t int_digits;
    if (*p == '0') {
      ++p;
      int_digits = 1;
    } else {
      int_digits = digits(w, nd, &fits);
    }
    int frac = 0;
    bool is_float = false;
    if (p < end && *p == '.') {
      ++p;
      is_float = true;
      const int nd0 = nd;
      if (digits(w, nd, &fits) == 0) return false;
      frac = nd - nd0;
    }
    long e10 = 0;
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      is_float = true;
      bool eneg = false;
      if (p < end && (*p == '+' || *p == '-')) eneg = *p++ == '-';
      if (p >= end || !digit(*p)) return false;
      while (p < end && digit(*p)) {
        if (e10 < 100000) e10 = e10 * 10 + (*p - '0');
        ++p;
      }
      if (eneg) e10 = -e10;
    }
    if (!is_float && int_digits > 18) return false;   // huge int literal: leave to Python
    if (!is_float && w == 0) {   // Python ints have no -0: int("-0") -> 0 -> +0.0
      *v = 0.0;
      return true;
    }
    const bool exact = fits;
    const long pw = e10 - frac;
    if (exact && w <= (uint64_t(1) << 53) && pw >= -22 && pw <= 22) {
      double d = static_cast<double>(w);
      d = pw >= 0 ? d * kPow10[pw] : d / kPow10[-pw];
      *v = neg ? -d : d;
      return true;
    }
    if (exact) {   // every digit is in w (<= 19 of them)
      *v = eisel_lemire(w, pw, neg);
      return true;
    }
    // more than 19 significant digits: correctly rounded strtod
    char small[128];
    const size_t n = static_cast<size_t>(p - s);
    std::string big;
    const char* txt;
    if (n < sizeof(small)) {
      std::memcpy(small, s, n);
      small[n] = 0;
      txt = small;
    } else {
      big.assign(s, n);
      txt = big.c_str();
    }
    char* q = nullptr;
    *v = std::strtod(txt, &q);
    return q == txt + n;
  }
};

}  // namespace

extern "C" int kf_parse_instances(const char* body, int64_t len, double* out, int64_t cap,
                                  int64_t* rows, int64_t* cols) {
  if (!body || len < 0 || !rows || !cols) return KF_FALLBACK;
  *rows = 0;
  *cols = 0;
  Scanner sc{body, body + len};
  sc.ws();
  if (!sc.eat('{')) return KF_FALLBACK;
  sc.ws();
  if (!sc.lit("\"instances\"", 11)) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat(':')) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat('[')) return KF_FALLBACK;
  int64_t r = 0, c = -1, n = 0;
  bool overflow = false;
  sc.ws();
  if (sc.p < sc.end && *sc.p == ']') return KF_FALLBACK;   // empty instances: the error path
  for (;;) {
    sc.ws();
    if (!sc.eat('[')) return KF_FALLBACK;
    int64_t k = 0;
    sc.ws();
    if (sc.p < sc.end && *sc.p == ']') return KF_FALLBACK;   // empty row
    for (;;) {
      sc.ws();
      double v;
      if (!sc.number(&v)) return KF_FALLBACK;
      if (n < cap) out[n] = v;
      else overflow = true;
      ++n;
      ++k;
      sc.ws();
      if (sc.eat(',')) continue;
      if (sc.eat(']')) break;
      return KF_FALLBACK;
    }
    if (c < 0) c = k;
    else if (k != c) return KF_FALLBACK;                     // ragged rows
    ++r;
    sc.ws();
    if (sc.eat(',')) continue;
    if (sc.eat(']')) break;
    return KF_FALLBACK;
  }
  sc.ws();
  if (!sc.eat('}')) return KF_FALLBACK;
  sc.ws();
  if (sc.p != sc.end) return KF_FALLBACK;
  *rows = r;
  *cols = c;
  return overflow ? KF_ERR_SPACE : KF_PARSED;
}

namespace {

// One row "[n, n, ...]" at sc.p: exactly want values into dst.
bool parse_row(Scanner& sc, double* dst, int64_t want) {
  if (!sc.eat('[')) return false;
  sc.ws();
  if (sc.p < sc.end && *sc.p == ']') return false;   // empty row
  int64_t k = 0;
  for (;;) {
    sc.ws();
    double v;
    if (k >= want || !sc.number(&v)) return false;   // too many values / not a number
    dst[k++] = v;
    sc.ws();
    if (sc.eat(',')) continue;
    if (sc.eat(']')) break;
    return false;
  }
  return k == want;
}

int64_t count_rows(const char* a, const char* b) {   // '[' = a row start in the rows region
  int64_t n = 0;
  while (a < b && (a = static_cast<const char*>(std::memchr(a, '[', static_cast<size_t>(b - a))))) {
    ++n;
    ++a;
  }
  return n;
}

const char* next_row(const char* a, const char* b) {
  const char* q = a < b ? static_cast<const char*>(std::memchr(a, '[', static_cast<size_t>(b - a)))
                        : nullptr;
  return q ? q : b;
}

}  // namespace

extern "C" int kf_parse_instances_mt(const char* body, int64_t len, double* out, int64_t cap,
                                     int64_t* rows, int64_t* cols, int32_t threads) {
  if (!body || len < 0 || !rows || !cols) return KF_FALLBACK;
  if (threads <= 1 || len < KF_MT_MIN_BYTES) return kf_parse_instances(body, len, out, cap, rows, cols);
  *rows = 0;
  *cols = 0;
  // the envelope: {"instances": [ ... ] } with whitespace anywhere
  Scanner sc{body, body + len};
  sc.ws();
  if (!sc.eat('{')) return KF_FALLBACK;
  sc.ws();
  if (!sc.lit("\"instances\"", 11)) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat(':')) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat('[')) return KF_FALLBACK;
  sc.ws();
  const char* p0 = sc.p;                             // the first row's '['
  const char* e = body + len;
  auto is_ws = [](char ch) { return ch == ' ' || ch == '\t' || ch == '\n' || ch == '\r'; };
  while (e > p0 && is_ws(e[-1])) --e;
  if (e <= p0 || e[-1] != '}') return KF_FALLBACK;
  --e;
  while (e > p0 && is_ws(e[-1])) --e;
  if (e <= p0 || e[-1] != ']') return KF_FALLBACK;
  --e;                                               // rows region [p0, e)
  if (p0 >= e || *p0 != '[') return KF_FALLBACK;
  // columns from the first row
  int64_t c = 0;
  {
    Scanner f{p0, e};
    if (!f.eat('[')) return KF_FALLBACK;
    for (;;) {
      f.ws();
      double v;
      if (!f.number(&v)) return KF_FALLBACK;
      ++c;
      f.ws();
      if (f.eat(',')) continue;
      if (f.eat(']')) break;
      return KF_FALLBACK;
    }
  }
  const int T = threads;
  std::vector<const char*> b(static_cast<size_t>(T) + 1);
  for (int i = 0; i <= T; ++i) b[i] = p0 + (e - p0) * i / T;
  std::vector<int64_t> n_rows(T, 0), r0(static_cast<size_t>(T) + 1, 0);
  std::vector<int> ok(T, 0);
  {
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i)
      th.emplace_back([&, i] { n_rows[i] = count_rows(b[i], b[i + 1]); });
    for (auto& t : th) t.join();
  }
  for (int i = 0; i < T; ++i) r0[i + 1] = r0[i] + n_rows[i];
  const int64_t R = r0[T];
  if (R * c > cap) {
    *rows = R;
    *cols = c;
    return KF_ERR_SPACE;
  }
  {
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i)
      th.emplace_back([&, i] {
        const char* start = next_row(b[i], b[i + 1]);
        const char* limit = i + 1 < T ? next_row(b[i + 1], e) : e;
        if (start >= limit) {   // no row starts in this slice
          ok[i] = n_rows[i] == 0;
          return;
        }
        Scanner s{start, e};
        int64_t r = r0[i];
        for (;;) {
          if (r >= r0[i + 1] || !parse_row(s, out + r * c, c)) return;
          ++r;
          s.ws();
          if (s.p == e) {   // the last row of the body: no comma after it
            ok[i] = limit == e && r == r0[i + 1];
            return;
          }
          if (!s.eat(',')) return;
          s.ws();
          if (s.p == limit) {   // the next slice's first row; a comma must be followed by a row,
            ok[i] = limit != e && r == r0[i + 1];   // so at the body's end it is a trailing comma
            return;
          }
          if (s.p > limit) return;
        }
      });
    for (auto& t : th) t.join();
  }
  for (int i = 0; i < T; ++i)
    if (!ok[i]) return KF_FALLBACK;
  *rows = R;
  *cols = c;
  return KF_PARSED;
}

// ------------------------------------------------------ lgbserver "inputs"
namespace {

// skip one JSON value of any kind at sc.p (a key the model does not read)
bool skip_value(Scanner& sc, int depth) {
  if (depth > 64) return false;
  sc.ws();
  if (sc.p >= sc.end) return false;
  const char c = *sc.p;
  if (c == '"') {
    ++sc.p;
    while (sc.p < sc.end && *sc.p != '"') {
      if (*sc.p == '\\') ++sc.p;
      ++sc.p;
    }
    return sc.eat('"');
  }
  if (c == '{' || c == '[') {
    const char close = c == '{' ? '}' : ']';
    ++sc.p;
    sc.ws();
    if (sc.eat(close)) return true;
    for (;;) {
      if (c == '{') {
        sc.ws();
        if (!skip_value(sc, depth + 1)) return false;   // the key
        sc.ws();
        if (!sc.eat(':')) return false;
      }
      if (!skip_value(sc, depth + 1)) return false;
      sc.ws();
      if (sc.eat(',')) continue;
      return sc.eat(close);
    }
  }
  if (sc.lit("true", 4) || sc.lit("false", 5) || sc.lit("null", 4)) return true;
  double v;
  return sc.number(&v);
}

}  // namespace

extern "C" int kf_parse_inputs(const char* body, int64_t len, const char* names,
                               const int32_t* name_offsets, int32_t n_names, double* out,
                               int64_t cap, int64_t* rows) {
  if (!body || len < 0 || !rows || n_names <= 0 || !names || !name_offsets) return KF_FALLBACK;
  *rows = 0;
  // the feature names, by text
  std::vector<std::pair<const char*, size_t>> nm(static_cast<size_t>(n_names));
  for (int32_t j = 0; j < n_names; ++j)
    nm[static_cast<size_t>(j)] = {names + name_offsets[j],
                                  static_cast<size_t>(name_offsets[j + 1] - name_offsets[j])};
  auto find = [&](const char* k, size_t n) -> int {
    for (int32_t j = 0; j < n_names; ++j)
      if (nm[static_cast<size_t>(j)].second == n &&
          std::memcmp(nm[static_cast<size_t>(j)].first, k, n) == 0)
        return j;
    return -1;
  };
  Scanner sc{body, body + len};
  sc.ws();
  if (!sc.eat('{')) return KF_FALLBACK;
  sc.ws();
  if (!sc.lit("\"inputs\"", 8)) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat(':')) return KF_FALLBACK;
  sc.ws();
  if (!sc.eat('[')) return KF_FALLBACK;
  sc.ws();
  if (sc.p < sc.end && *sc.p == ']') return KF_FALLBACK;   // no inputs: the error path
  int64_t R = 0;
  bool overflow = false;
  std::vector<std::vector<double>> col(static_cast<size_t>(n_names));
  std::vector<char> seen(static_cast<size_t>(n_names));
  for (;;) {   // one element of "inputs": an object of columns
    sc.ws();
    if (!sc.eat('{')) return KF_FALLBACK;
    std::fill(seen.begin(), seen.end(), 0);
    for (auto& v : col) v.clear();
    int64_t n = -1;   // this element's rows
    sc.ws();
    if (!sc.eat('}')) {
      for (;;) {
        sc.ws();
        if (!sc.eat('"')) return KF_FALLBACK;
        const char* k = sc.p;
        while (sc.p < sc.end && *sc.p != '"' && *sc.p != '\\') ++sc.p;
        if (sc.p >= sc.end || *sc.p == '\\') return KF_FALLBACK;   // escapes: json.loads
        const size_t kn = static_cast<size_t>(sc.p - k);
        ++sc.p;
        sc.ws();
        if (!sc.eat(':')) return KF_FALLBACK;
        sc.ws();
        const int j = find(k, kn);
        if (j < 0) {
          if (!skip_value(sc, 0)) return KF_FALLBACK;   // a key the model drops
        } else {
          if (seen[static_cast<size_t>(j)]) return KF_FALLBACK;   // duplicate: the last wins
          seen[static_cast<size_t>(j)] = 1;
          // a column: numbers with None beside them (None -> NaN), or all
          // booleans; anything else is pandas' (tree_model._numeric_column)
          if (!sc.eat('[')) return KF_FALLBACK;
          std::vector<double>& v = col[static_cast<size_t>(j)];
          int n_num = 0, n_bool = 0, n_none = 0;
          sc.ws();
          if (!sc.eat(']')) {
            for (;;) {
              sc.ws();
              double x;
              if (sc.lit("null", 4)) {
                ++n_none;
                x = std::nan("");
              } else if (sc.lit("true", 4)) {
                ++n_bool;
                x = 1.0;
              } else if (sc.lit("false", 5)) {
                ++n_bool;
                x = 0.0;
              } else if (sc.number(&x)) {
                ++n_num;
              } else {
                return KF_FALLBACK;
              }
              v.push_back(x);
              sc.ws();
              if (sc.eat(',')) continue;
              if (sc.eat(']')) break;
              return KF_FALLBACK;
            }
          }
          if (n_bool ? (n_num || n_none) : (n_num == 0 && !v.empty())) return KF_FALLBACK;
          const int64_t m = static_cast<int64_t>(v.size());
          if (n >= 0 && m != n) return KF_FALLBACK;   // columns of unequal length
          n = m;
        }
        sc.ws();
        if (sc.eat(',')) continue;
        if (sc.eat('}')) break;
        return KF_FALLBACK;
      }
    }
    if (n < 0) n = 0;
    for (int64_t r = 0; r < n; ++r)
      for (int32_t j = 0; j < n_names; ++j) {
        const int64_t at = (R + r) * n_names + j;
        const double x = seen[static_cast<size_t>(j)] ? col[static_cast<size_t>(j)][static_cast<size_t>(r)]
                                                      : std::nan("");
        if (at < cap) out[at] = x;
        else overflow = true;
      }
    R += n;
    sc.ws();
    if (sc.eat(',')) continue;
    if (sc.eat(']')) break;
    return KF_FALLBACK;
  }
  sc.ws();
  if (!sc.eat('}')) return KF_FALLBACK;
  sc.ws();
  if (sc.p != sc.end) return KF_FALLBACK;
  if (R == 0) return KF_FALLBACK;   // no rows: lgbserver's error
  *rows = R;
  return overflow ? KF_ERR_SPACE : KF_PARSED;
}

// --------------------------------------------------- V2 inference tensors
namespace {

// a JSON string of printable ASCII without escapes at sc.p ('"' included):
// its text is then the same after json.loads + json.dumps; anything else
// (escapes, controls, non-ASCII) is left to the application
bool plain_string(Scanner& sc, const char** s, int64_t* n) {
  if (!sc.eat('"')) return false;
  const char* a = sc.p;
  while (sc.p < sc.end && *sc.p != '"') {
    const unsigned char ch = static_cast<unsigned char>(*sc.p);
    if (ch < 0x20 || ch > 0x7E || ch == '\\') return false;
    ++sc.p;
  }
  if (sc.p >= sc.end) return false;
  *s = a - 1;
  *n = (sc.p - a) + 2;
  ++sc.p;
  return true;
}

// a Python int as a V2 shape entry: digits only (no sign, fraction, exponent)
bool shape_int(Scanner& sc, int64_t* v) {
  if (sc.p >= sc.end || !Scanner::digit(*sc.p)) return false;
  if (*sc.p == '0' && sc.end - sc.p > 1 && Scanner::digit(sc.p[1])) return false;   // "01"
  int64_t x = 0;
  int nd = 0;
  while (sc.p < sc.end && Scanner::digit(*sc.p)) {
    if (++nd > 12) return false;
    x = x * 10 + (*sc.p++ - '0');
  }
  *v = x;
  return true;
}

// "data": numbers, flat or one level of equal-length rows (np.asarray of
// it is then a 1- or 2-D array of the same values in the same order)
bool tensor_data(Scanner& sc, double* out, int64_t cap, int64_t* n) {
  if (!sc.eat('[')) return false;
  sc.ws();
  if (sc.p < sc.end && *sc.p == ']') return false;   // empty: the application
  const bool nested = sc.p < sc.end && *sc.p == '[';
  int64_t k = 0, width = -1;
  for (;;) {
    sc.ws();
    if (nested) {
      if (!sc.eat('[')) return false;
      int64_t w = 0;
      for (;;) {
        sc.ws();
        double v;
        if (!sc.number(&v)) return false;
        if (k < cap) out[k] = v;
        ++k;
        ++w;
        sc.ws();
        if (sc.eat(',')) continue;
        if (sc.eat(']')) break;
        return false;
      }
      if (width < 0) width = w;
      else if (w != width) return false;   // ragged: numpy's error
    } else {
      double v;
      if (!sc.number(&v)) return false;
      if (k < cap) out[k] = v;
      ++k;
    }
    sc.ws();
    if (sc.eat(',')) continue;
    if (sc.eat(']')) break;
    return false;
  }
  *n = k;
  return true;
}


// {"key": <value>} with one key: a non-negative int ("binary_data_size") or
// a boolean ("binary_data_output"); anything else is the application's
bool one_key_object(Scanner& sc, const char* key, size_t key_len, bool boolean, int64_t* v) {
  if (!sc.eat('{')) return false;
  sc.ws();
  if (!sc.lit(key, key_len)) return false;
  sc.ws();
  if (!sc.eat(':')) return false;
  sc.ws();
  if (boolean) {
    if (sc.lit("true", 4)) *v = 1;
    else if (sc.lit("false", 5)) *v = 0;
    else return false;
  } else if (!shape_int(sc, v)) {
    return false;
  }
  sc.ws();
  return sc.eat('}');
}

}  // namespace

extern "C" int kf_parse_v2_tensor(const char* body, int64_t len, int64_t head_len, double* out,
                                  int64_t cap, int64_t* rows, int64_t* cols, int32_t* datatype,
                                  int64_t* id_off, int64_t* id_len, int32_t* binary_output) {
  if (!body || len < 0 || head_len > len || !rows || !cols || !datatype || !id_off || !id_len ||
      !binary_output)
    return KF_FALLBACK;
  *rows = *cols = 0;
  *datatype = -1;
  *id_off = *id_len = 0;
  *binary_output = 0;
  const int64_t hl = head_len < 0 ? len : head_len;
  Scanner sc{body, body + hl};
  bool seen_inputs = false, seen_id = false, seen_params = false, overflow = false;
  int64_t shape[2] = {0, 0}, ndim = -1, count = -1, bsize = -1;
  sc.ws();
  if (!sc.eat('{')) return KF_FALLBACK;
  for (;;) {   // the request's keys: "inputs", "id" and "parameters" only
    sc.ws();
    if (sc.lit("\"inputs\"", 8)) {
      if (seen_inputs) return KF_FALLBACK;
      seen_inputs = true;
      sc.ws();
      if (!sc.eat(':')) return KF_FALLBACK;
      sc.ws();
      if (!sc.eat('[')) return KF_FALLBACK;
      sc.ws();
      if (!sc.eat('{')) return KF_FALLBACK;   // exactly one tensor
      bool s_name = false, s_shape = false, s_type = false, s_data = false, s_par = false;
      for (;;) {
        sc.ws();
        if (sc.lit("\"name\"", 6)) {
          if (s_name) return KF_FALLBACK;
          s_name = true;
          sc.ws();
          if (!sc.eat(':')) return KF_FALLBACK;
          sc.ws();
          const char* s;
          int64_t n;
          if (!plain_string(sc, &s, &n)) return KF_FALLBACK;
        } else if (sc.lit("\"shape\"", 7)) {
          if (s_shape) return KF_FALLBACK;
          s_shape = true;
          sc.ws();
          if (!sc.eat(':')) return KF_FALLBACK;
          sc.ws();
          if (!sc.eat('[')) return KF_FALLBACK;
          ndim = 0;
          for (;;) {
            sc.ws();
            int64_t d;
            if (ndim >= 2 || !shape_int(sc, &d)) return KF_FALLBACK;
            shape[ndim++] = d;
            sc.ws();
            if (sc.eat(',')) continue;
            if (sc.eat(']')) break;
            return KF_FALLBACK;
          }
        } else if (sc.lit("\"datatype\"", 10)) {
          if (s_type) return KF_FALLBACK;
          s_type = true;
          sc.ws();
          if (!sc.eat(':')) return KF_FALLBACK;
          sc.ws();
          if (sc.lit("\"FP32\"", 6)) *datatype = 0;
          else if (sc.lit("\"FP64\"", 6)) *datatype = 1;
          else return KF_FALLBACK;
        } else if (sc.lit("\"data\"", 6)) {
          if (s_data) return KF_FALLBACK;
          s_data = true;
          sc.ws();
          if (!sc.eat(':')) return KF_FALLBACK;
          sc.ws();
          if (!tensor_data(sc, out, cap, &count)) return KF_FALLBACK;
          if (count > cap) overflow = true;
        } else if (sc.lit("\"parameters\"", 12)) {   // binary tensor data
          if (s_par) return KF_FALLBACK;
          s_par = true;
          sc.ws();
          if (!sc.eat(':')) return KF_FALLBACK;
          sc.ws();
          if (!one_key_object(sc, "\"binary_data_size\"", 18, false, &bsize)) return KF_FALLBACK;
        } else {
          return KF_FALLBACK;
        }
        sc.ws();
        if (sc.eat(',')) continue;
        if (sc.eat('}')) break;
        return KF_FALLBACK;
      }
      // JSON data or binary data, not both
      if (!(s_shape && s_type && (s_data != (bsize >= 0)))) return KF_FALLBACK;
      sc.ws();
      if (!sc.eat(']')) return KF_FALLBACK;   // a second tensor: the application
    } else if (sc.lit("\"id\"", 4)) {
      if (seen_id) return KF_FALLBACK;
      seen_id = true;
      sc.ws();
      if (!sc.eat(':')) return KF_FALLBACK;
      sc.ws();
      const char* s;
      int64_t n;
      if (!plain_string(sc, &s, &n)) return KF_FALLBACK;
      *id_off = s - body;
      *id_len = n;
    } else if (sc.lit("\"parameters\"", 12)) {   // {"binary_data_output": bool}
      if (seen_params) return KF_FALLBACK;
      seen_params = true;
      sc.ws();
      if (!sc.eat(':')) return KF_FALLBACK;
      sc.ws();
      int64_t b = 0;
      if (!one_key_object(sc, "\"binary_data_output\"", 20, true, &b)) return KF_FALLBACK;
      *binary_output = static_cast<int32_t>(b);
    } else {
      return KF_FALLBACK;   // "outputs" and the rest: the application
    }
    sc.ws();
    if (sc.eat(',')) continue;
    if (sc.eat('}')) break;
    return KF_FALLBACK;
  }
  sc.ws();
  if (sc.p != sc.end || !seen_inputs || ndim < 1) return KF_FALLBACK;
  // np.asarray(data).size == prod(shape), reshaped; a [F] tensor is one row
  const int64_t r = ndim == 1 ? 1 : shape[0];
  const int64_t c = ndim == 1 ? shape[0] : shape[1];
  if (r <= 0 || c <= 0) return KF_FALLBACK;
  const int64_t tail = len - hl;
  if (bsize >= 0) {   // np.frombuffer of the tail: little-endian FP32 / FP64
    const int64_t es = *datatype == 0 ? 4 : 8;
    if (bsize != r * c * es || bsize != tail) return KF_FALLBACK;   // every byte one input's
    count = r * c;
    if (count > cap) {
      overflow = true;
    } else {
      const char* t = body + hl;
      for (int64_t i = 0; i < count; ++i) {
        if (es == 4) {
          float f;
          std::memcpy(&f, t + i * 4, 4);
          out[i] = f;
        } else {
          std::memcpy(&out[i], t + i * 8, 8);
        }
      }
    }
  } else if (tail != 0) {
    return KF_FALLBACK;   // binary data no input claims: the application's error
  }
  if (r * c != count) return KF_FALLBACK;
  *rows = r;
  *cols = c;
  return overflow ? KF_ERR_SPACE : KF_PARSED;
}
