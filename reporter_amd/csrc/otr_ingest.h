// otr_ingest.h — K11: probe text lines → windowed traces in HBM (include/otr.h
// otr_ingest).  One thread per line parses its fields; grouping by uuid, the stable time
// order and the inactivity windows (simple_reporter.py:146-160) are radix sorts, scans and
// scatters.  Number parsing reproduces Python's float() / int() exactly: decimals go
// through Clinger's fast path or the Eisel-Lemire algorithm (otr_pow5.h), both correctly
// rounded, and the rare inputs neither can decide are refused, never approximated.
//
// The parse functions are __host__ __device__ so that tests/ can check them on the CPU
// against Python itself (tools/libparsecheck.so, test infrastructure only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/otr.h"
#include "otr_pow5.h"

namespace otr {

#define OTR_HD __host__ __device__ inline

OTR_POW5_QUAL const double kP10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                       1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

OTR_HD bool py_space(uint8_t c) { return c == ' ' || (c >= 9 && c <= 13); }

OTR_HD void py_trim(const uint8_t* s, int64_t& b, int64_t& e) {
  while (b < e && py_space(s[b])) ++b;
  while (e > b && py_space(s[e - 1])) --e;
}

// value = ±w · 10^q; w holds the first 19 significant digits, `inexact` says a nonzero
// digit beyond them was dropped (then the value lies in (w, w + 1) · 10^q)
struct Dec {
  uint64_t w;
  int32_t q;
  bool neg;
  bool inexact;
};

// Python float() grammar for finite decimals: [ws][+-](d+[.d*]|.d+)[(e|E)[+-]d+][ws]
// (no inf/nan: a coordinate the reference could only carry as a non-number is refused)
OTR_HD bool parse_dec(const uint8_t* s, int64_t b, int64_t e, Dec& d) {
  py_trim(s, b, e);
  d.w = 0;
  d.q = 0;
  d.neg = false;
  d.inexact = false;
  if (b < e && (s[b] == '+' || s[b] == '-')) {
    d.neg = s[b] == '-';
    ++b;
  }
  int nd = 0, ndig = 0;
  int64_t q = 0;
  while (b < e && s[b] >= '0' && s[b] <= '9') {
    const uint32_t c = s[b++] - '0';
    ++ndig;
    if (nd < 19) {
      if (nd > 0 || c) {
        d.w = d.w * 10 + c;
        ++nd;
      }
    } else {
      ++q;
      d.inexact |= c != 0;
    }
  }
  if (b < e && s[b] == '.') {
    ++b;
    while (b < e && s[b] >= '0' && s[b] <= '9') {
      const uint32_t c = s[b++] - '0';
      ++ndig;
      if (nd < 19) {
        if (nd > 0 || c) {
          d.w = d.w * 10 + c;
          ++nd;
        }
        --q;
      } else {
        d.inexact |= c != 0;
      }
    }
  }
  if (ndig == 0) return false;
  if (b < e && (s[b] == 'e' || s[b] == 'E')) {
    ++b;
    bool eneg = false;
    if (b < e && (s[b] == '+' || s[b] == '-')) {
      eneg = s[b] == '-';
      ++b;
    }
    int ed = 0;
    int64_t x = 0;
    while (b < e && s[b] >= '0' && s[b] <= '9') {
      if (x < 1000000) x = x * 10 + (s[b] - '0');
      ++b;
      ++ed;
    }
    if (ed == 0) return false;
    q += eneg ? -x : x;
  }
  if (b != e) return false;
  d.q = q < -1000000 ? -1000000 : (q > 1000000 ? 1000000 : (int32_t)q);
  return true;
}

OTR_HD void mul_64x64(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
  const unsigned __int128 p = (unsigned __int128)a * b;
  hi = (uint64_t)(p >> 64);
  lo = (uint64_t)p;
}

// Eisel-Lemire (Lemire 2021, "Number Parsing at a Gigabyte per Second", §5-6): the
// binary64 nearest to w · 10^q (w > 0) from the 128-bit truncated product with 5^q.
// False only when the product's dropped bits leave the rounding undecided, which the
// paper shows cannot happen for q in [-27, 55].
OTR_HD bool eisel_lemire(uint64_t w, int32_t q, uint64_t& bits) {
  if (w == 0 || q < kPow5Min) {
    bits = 0;
    return true;
  }
  if (q > kPow5Max) {
    bits = 0x7FFull << 52;
    return true;
  }
  const int lz = __builtin_clzll(w);
  w <<= lz;
  const int row = q - kPow5Min;
  uint64_t hi, lo;
  mul_64x64(w, kPow5[row][0], hi, lo);
  if ((hi & 0x1FFu) == 0x1FFu) {  // the 55 bits kept might still change: add the next 64 bits
    uint64_t hi2, lo2;
    mul_64x64(w, kPow5[row][1], hi2, lo2);
    lo += hi2;
    if (hi2 > lo) ++hi;
  }
  if (lo == ~0ull && (q < -27 || q > 55)) return false;
  const int upper = (int)(hi >> 63);
  uint64_t m = hi >> (upper + 9);
  int32_t p2 = (int32_t)((((152170 + 65536) * q) >> 16) + 63) + upper - lz + 1023;
  if (p2 <= 0) {  // subnormal
    if (-p2 + 1 >= 64) {
      bits = 0;
      return true;
    }
    m >>= -p2 + 1;
    m += m & 1;
    m >>= 1;
    p2 = m < (1ull << 52) ? 0 : 1;
    bits = ((uint64_t)p2 << 52) | (m & ((1ull << 52) - 1));
    return true;
  }
  // exactly halfway between two doubles (possible only where 5^q is exact): round to even
  if (lo <= 1 && q >= -4 && q <= 23 && (m & 3) == 1 && (m << (upper + 9)) == hi) m &= ~1ull;
  m += m & 1;
  m >>= 1;
  if (m >= (2ull << 52)) {
    m = 1ull << 52;
    ++p2;
  }
  m &= ~(1ull << 52);
  if (p2 >= 0x7FF) {
    bits = 0x7FFull << 52;
    return true;
  }
  bits = ((uint64_t)p2 << 52) | m;
  return true;
}

OTR_HD double bits_double(uint64_t b) {
  union {
    uint64_t u;
    double d;
  } x;
  x.u = b;
  return x.d;
}
OTR_HD uint64_t double_bits(double v) {
  union {
    uint64_t u;
    double d;
  } x;
  x.d = v;
  return x.u;
}

// the double Python's float() returns for the decimal (false: undecidable here)
OTR_HD bool dec_to_double(const Dec& d, double& v) {
  uint64_t bits = 0;
  if (d.w == 0) {
    bits = 0;
  } else if (!d.inexact && d.w <= (1ull << 53) && d.q >= -22 && d.q <= 22) {
    // Clinger: w and 10^|q| are exact doubles, one correctly rounded operation
    const double x = (double)d.w;
    const double r = d.q < 0 ? x / kP10[-d.q] : x * kP10[d.q];
    v = d.neg ? -r : r;
    return true;
  } else if (!d.inexact) {
    if (!eisel_lemire(d.w, d.q, bits)) return false;
  } else {
    uint64_t b2 = 0;
    if (!eisel_lemire(d.w, d.q, bits) || !eisel_lemire(d.w + 1, d.q, b2) || bits != b2) return false;
  }
  v = bits_double(bits | (d.neg ? 1ull << 63 : 0ull));
  return true;
}

// Python int() of a byte range: [ws][+-]d+[ws] into int64 (strict: Long.parseLong, no
// whitespace); false on anything else or overflow
OTR_HD bool parse_int(const uint8_t* s, int64_t b, int64_t e, int64_t& out, bool strict = false) {
  if (!strict) py_trim(s, b, e);
  bool neg = false;
  if (b < e && (s[b] == '+' || s[b] == '-')) {
    neg = s[b] == '-';
    ++b;
  }
  if (b >= e) return false;
  uint64_t x = 0;
  for (; b < e; ++b) {
    if (s[b] < '0' || s[b] > '9') return false;
    if (x > (1ull << 63) / 10) return false;
    x = x * 10 + (s[b] - '0');
    if (x > (1ull << 63)) return false;
  }
  if (!neg && x == (1ull << 63)) return false;
  out = neg ? (int64_t)(0 - x) : (int64_t)x;
  return true;
}

// days from 1970-01-01 to y-m-d (proleptic Gregorian; Hinnant's days_from_civil)
OTR_HD int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

// simple_reporter.py:106-107 fast time: int() of tm[0:4], [5:7], [8:10], [11:13], [14:16],
// [17:19] (Python slices of the raw field, separators unchecked, the rest ignored), then
// calendar.timegm: datetime.date(year, month, 1) validates year and month, the other
// fields add linearly
OTR_HD int parse_ymdhms(const uint8_t* s, int64_t b, int64_t e, int64_t& t) {
  const int64_t n = e - b;
  const int lo[6] = {0, 5, 8, 11, 14, 17}, hi[6] = {4, 7, 10, 13, 16, 19};
  int64_t v[6];
  for (int k = 0; k < 6; ++k) {
    const int64_t pb = b + (lo[k] < n ? lo[k] : n), pe = b + (hi[k] < n ? hi[k] : n);
    if (!parse_int(s, pb, pe, v[k])) return OTR_INGEST_E_INT;
  }
  if (v[0] < 1 || v[0] > 9999 || v[1] < 1 || v[1] > 12) return OTR_INGEST_E_TIME;
  // |v[k]| < 10^4 for 4-char pieces, < 100 for 2-char ones: no overflow below
  const int64_t days = days_from_civil(v[0], v[1], 1) + v[2] - 1;
  t = ((days * 24 + v[3]) * 60 + v[4]) * 60 + v[5];
  return 0;
}

OTR_HD int digits_of(uint64_t w) {
  int n = 1;
  while (w >= 10) {
    w /= 10;
    ++n;
  }
  return n;
}

OTR_HD uint64_t pow10_u64(int k) {
  uint64_t r = 1;
  while (k-- > 0) r *= 10;
  return r;
}

// The coordinate simple_reporter.match() reads back after download() wrote it with
// Python 2 str() (simple_reporter.py:111): the decimal of 12 significant digits nearest
// to v (the double of d), re-parsed.  v's exact binary value decides the rounding; when
// v is the double nearest to the rounding midpoint the comparison is done exactly in
// 128-bit integers.  False: undecidable here (refused, never approximated).
OTR_HD bool py2_str_roundtrip(Dec d, double v, double& out) {
  if (d.w == 0) {
    out = v;
    return true;
  }
  if (!d.inexact)
    while (d.w % 10 == 0) {
      d.w /= 10;
      ++d.q;
    }
  const int nd = digits_of(d.w);
  if (nd <= 12 && !d.inexact) {
    out = v;  // the shortest 12-digit text is the input itself
    return true;
  }
  const int k = nd - 12;
  const uint64_t w12 = d.w / pow10_u64(k);
  // midpoint M = (10 w12 + 5) · 10^(q + k - 1) and its nearest double
  Dec mid;
  mid.w = w12 * 10 + 5;
  mid.q = d.q + k - 1;
  mid.neg = false;
  mid.inexact = false;
  double dm;
  if (!dec_to_double(mid, dm)) return false;
  const double av = v < 0 ? -v : v;
  int side;  // sign of |v| - M
  if (av != dm) {
    side = av < dm ? -1 : 1;
  } else {
    // exact: |v| = m · 2^e against M = N · 10^j, both scaled to integers
    const uint64_t vb = double_bits(av);
    const int ex = (int)((vb >> 52) & 0x7FF);
    if (ex == 0 || ex == 0x7FF) return false;
    const uint64_t m = (vb & ((1ull << 52) - 1)) | (1ull << 52);
    const int e2 = ex - 1075;
    const int j = mid.q;
    if (j >= 0 || -j > 27 || e2 >= 0) return false;
    // |v| < M  ⟺  m · 5^-j · 2^(e2 - j) < N
    unsigned __int128 lhs = m;
    for (int i = 0; i < -j; ++i) lhs *= 5;
    unsigned __int128 rhs = mid.w;
    const int sh = e2 - j;
    if (sh >= 0) {
      if (sh > 10) return false;  // lhs < 2^116: keep the shift inside 128 bits
      lhs <<= sh;
    } else {
      if (-sh > 83) return false;  // N < 2^44
      rhs <<= -sh;
    }
    side = lhs < rhs ? -1 : (lhs > rhs ? 1 : 0);
  }
  Dec r;
  r.w = side < 0 ? w12 : (side > 0 ? w12 + 1 : w12 + (w12 & 1));  // exact tie: half even
  r.q = d.q + k;
  r.neg = d.neg;
  r.inexact = false;
  return dec_to_double(r, out);
}

OTR_HD uint64_t uuid_hash(const uint8_t* s, int64_t b, int64_t e) {
  uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a, then a splitmix64 finaliser
  for (; b < e; ++b) h = (h ^ s[b]) * 0x100000001b3ull;
  h ^= h >> 30;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 27;
  h *= 0x94d049bb133111ebull;
  return h ^ (h >> 31);
}

// ---- kernels --------------------------------------------------------------------------
#ifndef OTR_INGEST_PARSE_ONLY

struct IngestFmt {
  int rules, sep, tfmt, use_bbox;
  int idx[5];  // uuid, time, lat, lon, accuracy field positions
  double bbox[4];
};

struct IngestLines {
  const uint8_t* text;
  int64_t len;
  const int64_t* nl;  // positions of '\n'
  int64_t n_nl, n_lines;
  uint64_t* hash;
  int64_t* uoff;
  int32_t* ulen;
  int64_t* time;
  double* lat;
  double* lon;
  float* acc;
  int64_t* keep;
  unsigned long long* bad;  // min over rejected lines of (line << 8 | reason)
};

// newline counts per 16-byte chunk (text padded to a multiple of 16 with zeros)
__global__ void k_nl_count(const uint4* text, int64_t n_chunks, int64_t* cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chunks) return;
  const uint4 v = text[c];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  int n = 0;
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = w[k] ^ 0x0A0A0A0Au;  // zero bytes where '\n' (exact per-byte test)
    n += __popc(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu));
  }
  cnt[c] = n;
}

__global__ void k_nl_write(const uint4* text, int64_t n_chunks, const int64_t* scan, int64_t* nl) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chunks) return;
  int64_t o = c ? scan[c - 1] : 0;
  if (scan[c] == o) return;
  const uint4 v = text[c];
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (int k = 0; k < 16; ++k)
    if (((w[k >> 2] >> (8 * (k & 3))) & 0xFF) == 0x0A) nl[o++] = 16 * c + k;
}

__device__ inline void ingest_reject(const IngestLines& L, int64_t line, int reason) {
  atomicMin(L.bad, ((unsigned long long)line << 8) | (unsigned)reason);
}

// one thread per line: fields, numbers, bbox (include/otr.h otr_ingest for the rules)
__global__ void k_ingest_parse(IngestLines L, IngestFmt f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= L.n_lines) return;
  const uint8_t* s = L.text;
  int64_t b = i ? L.nl[i - 1] + 1 : 0;
  int64_t e = i < L.n_nl ? L.nl[i] : L.len;
  L.keep[i] = 0;
  int64_t fb[5] = {0, 0, 0, 0, 0}, fe[5] = {0, 0, 0, 0, 0};
  bool have[5] = {false, false, false, false, false};
  const bool shard = f.rules == OTR_INGEST_SHARD;
  if (shard) py_trim(s, b, e);  // line.strip() (:140)
  const uint8_t sep = shard ? (uint8_t)',' : (uint8_t)f.sep;
  int nf = 0, last_nonempty = -1;
  int64_t st = b;
  for (int64_t p = b; p <= e; ++p) {
    if (p == e || s[p] == sep) {
      for (int k = 0; k < 5; ++k)
        if ((shard ? k : f.idx[k]) == nf) {
          fb[k] = st;
          fe[k] = p;
          have[k] = true;
        }
      if (p > st) last_nonempty = nf;
      ++nf;
      st = p + 1;
    }
  }
  // SHARD: tuple unpack of exactly 5; RAW: IndexError; JAVA: String.split drops the
  // trailing empty fields before indexing
  const int n_avail = f.rules == OTR_INGEST_JAVA_SV ? last_nonempty + 1 : nf;
  bool ok = shard ? nf == 5 : true;
  for (int k = 0; k < 5; ++k) ok = ok && have[k] && (shard ? k : f.idx[k]) < n_avail;
  if (!ok) {
    ingest_reject(L, i, OTR_INGEST_E_FIELDS);
    return;
  }
  // coordinates
  Dec dla, dlo;
  double la = 0, lo = 0;
  if (!parse_dec(s, fb[2], fe[2], dla) || !parse_dec(s, fb[3], fe[3], dlo)) {
    ingest_reject(L, i, OTR_INGEST_E_FLOAT);
    return;
  }
  if (!dec_to_double(dla, la) || !dec_to_double(dlo, lo)) {
    ingest_reject(L, i, OTR_INGEST_E_PRECISION);
    return;
  }
  if (f.rules == OTR_INGEST_RAW && f.use_bbox &&
      (la < f.bbox[0] || la > f.bbox[2] || lo < f.bbox[1] || lo > f.bbox[3]))
    return;  // skipped before time and accuracy are looked at (:103-105)
  if (!(la - la == 0.0) || !(lo - lo == 0.0)) {
    ingest_reject(L, i, OTR_INGEST_E_FLOAT);
    return;
  }
  // time
  int64_t t = 0;
  if (f.rules != OTR_INGEST_SHARD && f.tfmt == OTR_TIME_YMDHMS) {
    const int r = parse_ymdhms(s, fb[1], fe[1], t);
    if (r) {
      ingest_reject(L, i, r);
      return;
    }
  } else if (!parse_int(s, fb[1], fe[1], t, f.rules == OTR_INGEST_JAVA_SV)) {
    ingest_reject(L, i, OTR_INGEST_E_INT);
    return;
  }
  // accuracy
  int64_t a = 0;
  if (shard) {
    if (!parse_int(s, fb[4], fe[4], a)) {
      ingest_reject(L, i, OTR_INGEST_E_INT);
      return;
    }
  } else {
    Dec da;
    double av = 0;
    if (!parse_dec(s, fb[4], fe[4], da) || !dec_to_double(da, av) || !(av - av == 0.0)) {
      ingest_reject(L, i, OTR_INGEST_E_ACCURACY);
      return;
    }
    if (f.rules == OTR_INGEST_RAW) {
      const double c = ceil(av);  // min(int(math.ceil(float(acc))), 1000)
      if (c < -16777216.0) {
        ingest_reject(L, i, OTR_INGEST_E_ACCURACY);
        return;
      }
      a = c > 1000.0 ? 1000 : (int64_t)c;
    } else {
      const float af = (float)av;  // (int)Math.ceil(float): saturating cast
      const double c = ceil((double)af);
      a = c >= 2147483647.0 ? 2147483647 : (c <= -2147483648.0 ? -2147483647 - 1 : (int64_t)c);
    }
  }
  if (a > 16777216 || a < -16777216) {
    ingest_reject(L, i, OTR_INGEST_E_ACCURACY);
    return;
  }
  // coordinates as the matcher sees them
  if (f.rules == OTR_INGEST_RAW) {
    double la2, lo2;
    if (!py2_str_roundtrip(dla, la, la2) || !py2_str_roundtrip(dlo, lo, lo2)) {
      ingest_reject(L, i, OTR_INGEST_E_PRECISION);
      return;
    }
    la = la2;
    lo = lo2;
  } else if (f.rules == OTR_INGEST_JAVA_SV) {
    la = (double)(float)la;
    lo = (double)(float)lo;
  }
  // uuid: the shard round trip strips its leading whitespace and cannot carry ','
  int64_t ub = fb[0], ue = fe[0];
  if (f.rules == OTR_INGEST_RAW) {
    while (ub < ue && py_space(s[ub])) ++ub;
    for (int64_t p = ub; p < ue; ++p)
      if (s[p] == ',') {
        ingest_reject(L, i, OTR_INGEST_E_UUID);
        return;
      }
  }
  L.hash[i] = uuid_hash(s, ub, ue);
  L.uoff[i] = ub;
  L.ulen[i] = (int32_t)(ue - ub);
  L.time[i] = t;
  L.lat[i] = la;
  L.lon[i] = lo;
  L.acc[i] = (float)a;
  L.keep[i] = 1;
}

template <class T>
__global__ void k_gather_by(const T* src, const int32_t* idx, int64_t n, T* dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

__global__ void k_scatter_index32(const int64_t* flag, const int64_t* pos, int64_t n, int32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) out[pos[i] - 1] = (int32_t)i;
}

// uuid groups over lines sorted by (hash, line): heads, and a string check of every
// equal-hash neighbour (a collision is refused, never merged)
__global__ void k_group_heads(const uint64_t* hash, const int32_t* line, int64_t m, const int64_t* uoff,
                              const int32_t* ulen, const uint8_t* text, int64_t* head, unsigned long long* bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  if (i == 0 || hash[i] != hash[i - 1]) {
    head[i] = 1;
    return;
  }
  head[i] = 0;
  const int32_t a = line[i - 1], c = line[i];
  bool same = ulen[a] == ulen[c];
  for (int32_t k = 0; same && k < ulen[a]; ++k) same = text[uoff[a] + k] == text[uoff[c] + k];
  if (!same) atomicMin(bad, ((unsigned long long)c << 8) | OTR_INGEST_E_COLLISION);
}

// first line of each group (sorted by line within a hash), then per line its group's
// first line: the trace order key
__global__ void k_group_first(const int64_t* head, const int64_t* gid, const int32_t* line, int64_t m,
                              int32_t* gfirst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m && head[i]) gfirst[gid[i] - 1] = line[i];
}
__global__ void k_group_key(const int64_t* gid, const int32_t* line, int64_t m, const int32_t* gfirst,
                            uint32_t* key_of_line) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < m) key_of_line[line[i]] = (uint32_t)gfirst[gid[i] - 1];
}

// window heads in final (group, time, line) order: new uuid or a gap > inactivity (:150-152)
__global__ void k_win_heads(const int32_t* perm, int64_t m, const uint32_t* gkey, const int64_t* time,
                            int64_t inactivity, int64_t* head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  if (i == 0) {
    head[i] = 1;
    return;
  }
  const int32_t a = perm[i - 1], c = perm[i];
  const __int128 gap = (__int128)time[c] - (__int128)time[a];
  head[i] = gkey[a] != gkey[c] || gap > (__int128)inactivity;
}

// per window: its length if kept (>= 2 points, :155-158) and a kept flag
__global__ void k_win_len(const int64_t* ws, int64_t n_win, int64_t m, int64_t* klen, int64_t* kflag) {
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= n_win) return;
  const int64_t len = (w + 1 < n_win ? ws[w + 1] : m) - ws[w];
  klen[w] = len >= 2 ? len : 0;
  kflag[w] = len >= 2;
}

struct IngestOut {
  int64_t* trace_off;
  double* lat;
  double* lon;
  int64_t* time;
  float* acc;
  uint8_t* mode;
  int64_t* uoff;
  int32_t* ulen;
};

__global__ void k_win_emit(const int32_t* perm, int64_t m, const int64_t* wid, const int64_t* ws, const int64_t* klen,
                           const int64_t* poff, const int64_t* tpos, int32_t n_traces, IngestLines L, uint8_t mode,
                           IngestOut o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const int64_t w = wid[i] - 1;
  const int64_t len = klen[w];
  if (len == 0) return;
  const int64_t t = tpos[w] - 1;
  const int64_t base = poff[w] - len;
  const int64_t k = base + (i - ws[w]);
  const int32_t ln = perm[i];
  o.lat[k] = L.lat[ln];
  o.lon[k] = L.lon[ln];
  o.time[k] = L.time[ln];
  o.acc[k] = L.acc[ln];
  if (i == ws[w]) {
    o.trace_off[t] = base;
    o.mode[t] = mode;
    o.uoff[t] = L.uoff[ln];
    o.ulen[t] = L.ulen[ln];
    if (t == n_traces - 1) o.trace_off[n_traces] = poff[w];
  }
}

#endif  // OTR_INGEST_PARSE_ONLY
}  // namespace otr
