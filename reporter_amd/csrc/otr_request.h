// otr_request.h — single-pass scanner for the POST /report body straight into SoA
// (no DOM), and Python-repr float output for the response bodies.
//
// Request body: Batch.java:56-65 builds {"uuid":..,"match_options":{"mode":..,
// "report_levels":[..],"transition_levels":[..]},"trace":[{lat,lon,time[,accuracy]},..]}
// (Point.java:59-65); reporter_service.py:209-235 validates it in this order:
//   uuid present and not null (:217-219) → trace[1] exists (:222-225) →
//   match_options.report_levels (:228-231) → match_options.transition_levels (:232-235)
// and every failure past that point is Match() raising (→ 500, :244-245).
// Duplicate keys resolve to the last occurrence, as Python's json.loads does.
//
// Response numbers: json.dumps (reporter_service.py:243) prints floats with repr():
// the shortest round-trip digits, fixed notation for decimal exponents -4..15 and
// d.ddde±XX otherwise, "NaN"/"Infinity" for the non-finite values.
#pragma once
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace otrreq {

// match_options numeric overrides (meili parameter names, Dockerfile:14-17,42-49)
enum Override {
  OV_SIGMA_Z = 0,
  OV_BETA,
  OV_ROUTE_FACTOR,
  OV_BREAKAGE,
  OV_INTERPOLATION,
  OV_SEARCH_RADIUS,
  OV_MAX_SEARCH_RADIUS,
  OV_GPS_ACCURACY,
  OV_MAX_CANDIDATES,
  OV_TIME_FACTOR,
  OV_TURN_PENALTY,
  OV_COUNT
};
static const char* const kOverrideNames[OV_COUNT] = {
    "sigma_z",         "beta",          "max_route_distance_factor", "breakage_distance", "interpolation_distance",
    "search_radius",   "max_search_radius", "gps_accuracy",          "max_candidates",
    "max_route_time_factor", "turn_penalty_factor"};

struct Request {
  int code = 0;  // 0 = valid; else 400 (request) or 500 (what Match() would raise on)
  std::string err;
  bool has_uuid = false;
  std::string uuid;
  bool trace_array = false;
  size_t trace_items = 0;
  size_t trace_str_chars = 0;  // "trace" given as a string: trace['trace'][1] indexes its characters
  bool points_ok = true;  // every trace item is an object with numeric lat, lon, time
  bool rl_array = false, tl_array = false;
  uint32_t rl = 0, tl = 0;
  uint8_t mode = 0;        // 0 auto, 1 bicycle, 2 pedestrian
  uint32_t ov_mask = 0;    // bit k: override k present
  double ov[OV_COUNT] = {0};
  bool any_acc = false;
  std::vector<double> lat, lon;
  std::vector<int64_t> time;
  std::vector<float> acc;
};

inline int mode_index(const std::string& m) {
  if (m == "bicycle") return 1;
  if (m == "pedestrian" || m == "foot") return 2;
  return 0;  // auto and the other motor modes share auto access
}

class Scanner {
 public:
  Scanner(const char* s, size_t n) : p_(s), e_(s + n) {}

  // Fills *r.  Report bodies (match_only = false) are validated as handle_request does
  // (400 for the request errors, 500 for what Match() would raise on).  Match() bodies
  // (match_only = true) need only a trace array of complete points; any failure is 500.
  bool request(Request* r, bool match_only = false) {
    match_only_ = match_only;
    ws();
    if (p_ >= e_) return bad(r, "No json provided");
    if (*p_ != '{') {
      if (!skip(0)) return bad(r, err_.c_str());
      ws();
      if (p_ != e_) return bad(r, "Extra data");
      if (match_only_) return bad(r, "trace is required");
      return bad(r, "uuid is required");  // not an object: trace.get('uuid') has nothing to give
    }
    ++p_;
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
      return finish(r);
    }
    for (;;) {
      std::string key;
      ws();
      if (!string(&key)) return bad(r, err_.c_str());
      ws();
      if (p_ >= e_ || *p_ != ':') return bad(r, "Expecting ':' delimiter");
      ++p_;
      ws();
      bool ok;
      if (key == "uuid") ok = uuid(r);
      else if (key == "trace") ok = trace(r);
      else if (key == "match_options") ok = options(r);
      else ok = skip(0);
      if (!ok) return bad(r, err_.c_str());
      ws();
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < e_ && *p_ == '}') {
        ++p_;
        break;
      }
      return bad(r, "Expecting ',' delimiter");
    }
    return finish(r);
  }

 private:
  const char* p_;
  const char* e_;
  std::string err_;
  bool match_only_ = false;

  bool bad(Request* r, const char* m) {
    r->code = match_only_ ? 500 : 400;
    r->err = (m && *m) ? m : "invalid JSON";
    return false;
  }
  bool finish(Request* r) {
    ws();
    if (p_ != e_ && *p_ != '\0') return bad(r, "Extra data");
    if (match_only_) {
      if (!r->trace_array || !r->points_ok) {
        r->code = 500;
        r->err = "trace must be a non zero length array of object each of which must have at least lat, lon and time";
        return false;
      }
      r->code = 0;
      return true;
    }
    // validation order of reporter_service.py:216-235
    if (!r->has_uuid) return bad(r, "uuid is required");
    if ((!r->trace_array || r->trace_items < 2) && r->trace_str_chars < 2)
      return bad(r, "trace must be a non zero length array of object each of which must have at least lat, lon "
                    "and time");
    if (!r->rl_array) return bad(r, "match_options must include report_levels array");
    if (!r->tl_array) return bad(r, "match_options must include transition_levels array");
    if (!r->points_ok || !r->trace_array) {
      r->code = 500;
      r->err = "trace must be a non zero length array of object each of which must have at least lat, lon and time";
      return false;
    }
    r->code = 0;
    return true;
  }
  bool fail(const char* m) {
    if (err_.empty()) err_ = m;
    return false;
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  static void put_utf8(std::string* o, uint32_t c) {
    if (c < 0x80) {
      o->push_back((char)c);
    } else if (c < 0x800) {
      o->push_back((char)(0xC0 | (c >> 6)));
      o->push_back((char)(0x80 | (c & 0x3F)));
    } else if (c < 0x10000) {
      o->push_back((char)(0xE0 | (c >> 12)));
      o->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      o->push_back((char)(0x80 | (c & 0x3F)));
    } else {
      o->push_back((char)(0xF0 | (c >> 18)));
      o->push_back((char)(0x80 | ((c >> 12) & 0x3F)));
      o->push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      o->push_back((char)(0x80 | (c & 0x3F)));
    }
  }
  bool hex4(uint32_t* v) {
    if (e_ - p_ < 4) return fail("Invalid \\uXXXX escape");
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = p_[k];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return fail("Invalid \\uXXXX escape");
    }
    p_ += 4;
    *v = x;
    return true;
  }
  // JSON string at p_ (opening quote); out == nullptr skips it
  bool string(std::string* out) {
    if (p_ >= e_ || *p_ != '"') return fail("Expecting property name enclosed in double quotes");
    ++p_;
    for (;;) {
      const char* q = p_;
      while (q < e_ && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
      if (out) out->append(p_, q);
      p_ = q;
      if (p_ >= e_) return fail("Unterminated string");
      const char c = *p_++;
      if (c == '"') return true;
      if (c != '\\') return fail("Invalid control character in string");
      if (p_ >= e_) return fail("Unterminated string");
      const char x = *p_++;
      char ch = 0;
      switch (x) {
        case '"': ch = '"'; break;
        case '\\': ch = '\\'; break;
        case '/': ch = '/'; break;
        case 'b': ch = '\b'; break;
        case 'f': ch = '\f'; break;
        case 'n': ch = '\n'; break;
        case 'r': ch = '\r'; break;
        case 't': ch = '\t'; break;
        case 'u': {
          uint32_t u;
          if (!hex4(&u)) return false;
          if (u >= 0xD800 && u < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            const char* save = p_;
            p_ += 2;
            uint32_t lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
            else p_ = save;
          }
          if (out) put_utf8(out, u);
          continue;
        }
        default: return fail("Invalid \\escape");
      }
      if (out) out->push_back(ch);
    }
  }
  // JSON number (plus NaN / Infinity / -Infinity, which Python's json accepts)
  bool number(double* d, int64_t* i, bool* is_int) {
    const char* s = p_;
    if (e_ - p_ >= 3 && !strncmp(p_, "NaN", 3)) {
      p_ += 3;
      *d = NAN;
      *is_int = false;
      return true;
    }
    const bool neg = p_ < e_ && *p_ == '-';
    const char* q = neg ? p_ + 1 : p_;
    if (e_ - q >= 8 && !strncmp(q, "Infinity", 8)) {
      p_ = q + 8;
      *d = neg ? -INFINITY : INFINITY;
      *is_int = false;
      return true;
    }
    if (q >= e_ || *q < '0' || *q > '9') return fail("Expecting value");
    if (*q == '0') ++q;
    else
      while (q < e_ && *q >= '0' && *q <= '9') ++q;
    bool integral = true;
    if (q < e_ && *q == '.') {
      ++q;
      if (q >= e_ || *q < '0' || *q > '9') return fail("Expecting value");
      while (q < e_ && *q >= '0' && *q <= '9') ++q;
      integral = false;
    }
    if (q < e_ && (*q == 'e' || *q == 'E')) {
      ++q;
      if (q < e_ && (*q == '+' || *q == '-')) ++q;
      if (q >= e_ || *q < '0' || *q > '9') return fail("Expecting value");
      while (q < e_ && *q >= '0' && *q <= '9') ++q;
      integral = false;
    }
    p_ = q;
    if (integral) {
      auto r = std::from_chars(s, q, *i);
      if (r.ec == std::errc()) {
        *d = (double)*i;
        *is_int = true;
        return true;
      }
    } else if (fast_decimal(s, q, d)) {
      *is_int = false;
      return true;
    }
    // correctly rounded, as Python's float(str)
    auto r = std::from_chars(s, q, *d);
    if (r.ec != std::errc() && r.ec != std::errc::result_out_of_range) return fail("Expecting value");
    if (r.ec == std::errc::result_out_of_range) *d = strtod(std::string(s, q).c_str(), nullptr);
    *is_int = false;
    return true;
  }
  // Clinger's fast path: [-]digits.digits with a mantissa below 2^53 and at most 22
  // fraction digits is M / 10^k with both operands exact, so the one IEEE division is
  // the correctly rounded value (what Python's float(str) returns).
  static bool fast_decimal(const char* s, const char* e, double* d) {
    static const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                      1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    const bool neg = *s == '-';
    if (neg) ++s;
    uint64_t m = 0;
    int nd = 0, frac = -1;
    for (const char* q = s; q < e; ++q) {
      if (*q == '.') {
        frac = 0;
        continue;
      }
      if (*q < '0' || *q > '9') return false;  // exponent: slow path
      if (++nd > 17) return false;
      m = m * 10 + (uint64_t)(*q - '0');
      if (frac >= 0) ++frac;
    }
    if (frac < 0 || frac > 22 || m >= (1ull << 53)) return false;
    const double v = (double)m / kPow10[frac];
    *d = neg ? -v : v;
    return true;
  }
  bool literal(const char* w) {
    const size_t n = strlen(w);
    if ((size_t)(e_ - p_) < n || strncmp(p_, w, n)) return fail("Expecting value");
    p_ += n;
    return true;
  }
  // any value
  bool skip(int depth) {
    if (depth > 256) return fail("JSON nested too deeply");
    ws();
    if (p_ >= e_) return fail("Expecting value");
    const char c = *p_;
    if (c == '"') return string(nullptr);
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      ++p_;
      ws();
      if (p_ < e_ && *p_ == close) {
        ++p_;
        return true;
      }
      for (;;) {
        ws();
        if (c == '{') {
          if (!string(nullptr)) return false;
          ws();
          if (p_ >= e_ || *p_ != ':') return fail("Expecting ':' delimiter");
          ++p_;
        }
        if (!skip(depth + 1)) return false;
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == close) {
          ++p_;
          return true;
        }
        return fail("Expecting ',' delimiter");
      }
    }
    if (c == 't') return literal("true");
    if (c == 'f') return literal("false");
    if (c == 'n') return literal("null");
    double d;
    int64_t i;
    bool ii;
    return number(&d, &i, &ii);
  }
  bool is_number_start() const {
    return p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '-' || *p_ == 'N' || *p_ == 'I');
  }
  bool uuid(Request* r) {
    r->uuid.clear();
    if (p_ < e_ && *p_ == 'n') {
      r->has_uuid = false;  // null is "not given" (trace.get('uuid') is None)
      return literal("null");
    }
    r->has_uuid = true;
    if (p_ < e_ && *p_ == '"') return string(&r->uuid);
    return skip(0);
  }
  bool trace(Request* r) {
    r->lat.clear();
    r->lon.clear();
    r->time.clear();
    r->acc.clear();
    r->any_acc = false;
    r->points_ok = true;
    r->trace_items = 0;
    r->trace_str_chars = 0;
    r->trace_array = p_ < e_ && *p_ == '[';
    if (r->trace_array) {  // ~40 bytes per point in Batch.java's layout
      const size_t est = (size_t)(e_ - p_) / 40 + 4;
      r->lat.reserve(est);
      r->lon.reserve(est);
      r->time.reserve(est);
      r->acc.reserve(est);
    }
    if (!r->trace_array) {
      if (p_ < e_ && *p_ == '"') {
        std::string s;
        if (!string(&s)) return false;
        for (unsigned char c : s) r->trace_str_chars += (c & 0xC0) != 0x80;  // code points
        return true;
      }
      return skip(0);
    }
    ++p_;
    ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
      return true;
    }
    for (;;) {
      ws();
      ++r->trace_items;
      if (!point(r)) return false;
      ws();
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < e_ && *p_ == ']') {
        ++p_;
        return true;
      }
      return fail("Expecting ',' delimiter");
    }
  }
  // key of a trace point: 0 lat, 1 lon, 2 time, 3 accuracy, -1 other, -2 error.
  // Escape-free keys are matched in place (the common case: no allocation).
  int point_key() {
    if (p_ < e_ && *p_ == '"') {
      const char* q = p_ + 1;
      while (q < e_ && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
      if (q < e_ && *q == '"') {
        const size_t n = (size_t)(q - p_ - 1);
        const char* k = p_ + 1;
        p_ = q + 1;
        if (n == 3 && k[0] == 'l' && k[1] == 'a' && k[2] == 't') return 0;
        if (n == 3 && k[0] == 'l' && k[1] == 'o' && k[2] == 'n') return 1;
        if (n == 4 && !memcmp(k, "time", 4)) return 2;
        if (n == 8 && !memcmp(k, "accuracy", 8)) return 3;
        return -1;
      }
    }
    std::string key;
    if (!string(&key)) return -2;
    return key == "lat" ? 0 : key == "lon" ? 1 : key == "time" ? 2 : key == "accuracy" ? 3 : -1;
  }
  bool point(Request* r) {
    if (p_ >= e_ || *p_ != '{') {
      r->points_ok = false;
      return skip(1);
    }
    ++p_;
    double lat = 0, lon = 0, acc = 0, tm = 0;
    int64_t ti = 0;
    bool have_lat = false, have_lon = false, have_time = false, have_acc = false, t_int = false;
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
    } else {
      for (;;) {
        ws();
        const int which = point_key();
        if (which == -2) return false;
        ws();
        if (p_ >= e_ || *p_ != ':') return fail("Expecting ':' delimiter");
        ++p_;
        ws();
        if (which >= 0 && is_number_start()) {
          double d;
          int64_t i;
          bool ii;
          if (!number(&d, &i, &ii)) return false;
          if (which == 0) lat = d, have_lat = true;
          else if (which == 1) lon = d, have_lon = true;
          else if (which == 2) tm = d, ti = i, t_int = ii, have_time = true;
          else acc = d, have_acc = true;
        } else {
          if (which == 0) have_lat = false;
          else if (which == 1) have_lon = false;
          else if (which == 2) have_time = false;
          else if (which == 3) have_acc = false;
          if (!skip(1)) return false;
        }
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == '}') {
          ++p_;
          break;
        }
        return fail("Expecting ',' delimiter");
      }
    }
    if (!have_lat || !have_lon || !have_time) {
      r->points_ok = false;
      return true;
    }
    r->lat.push_back(lat);
    r->lon.push_back(lon);
    r->time.push_back(t_int ? ti : (int64_t)std::floor(tm));
    r->acc.push_back(have_acc ? (float)acc : -1.f);
    r->any_acc = r->any_acc || have_acc;
    return true;
  }
  // set(match_options[...]) (reporter_service.py:229,233) accepts any iterable: a
  // string or an object iterates to strings, which never equal a level; numbers and
  // booleans compare by value (1.0 == 1, True == 1)
  bool levels(uint32_t* mask, bool* is_array) {
    *mask = 0;
    *is_array = p_ < e_ && (*p_ == '[' || *p_ == '"' || *p_ == '{');
    if (p_ >= e_ || *p_ != '[') return skip(1);
    ++p_;
    ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
      return true;
    }
    for (;;) {
      ws();
      if (is_number_start()) {
        double d;
        int64_t i;
        bool ii;
        if (!number(&d, &i, &ii)) return false;
        const int64_t l = ii ? i : (int64_t)d;
        if (l >= 0 && l < 32 && (ii || d == (double)l)) *mask |= 1u << l;
      } else if (p_ < e_ && (*p_ == 't' || *p_ == 'f')) {
        const bool t = *p_ == 't';
        if (!literal(t ? "true" : "false")) return false;
        *mask |= t ? 2u : 1u;
      } else if (!skip(2)) {
        return false;
      }
      ws();
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < e_ && *p_ == ']') {
        ++p_;
        return true;
      }
      return fail("Expecting ',' delimiter");
    }
  }
  bool options(Request* r) {
    r->rl_array = r->tl_array = false;
    r->rl = r->tl = 0;
    r->mode = 0;
    r->ov_mask = 0;
    if (p_ >= e_ || *p_ != '{') return skip(0);
    ++p_;
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
      return true;
    }
    for (;;) {
      std::string key;
      ws();
      if (!string(&key)) return false;
      ws();
      if (p_ >= e_ || *p_ != ':') return fail("Expecting ':' delimiter");
      ++p_;
      ws();
      bool ok = true;
      if (key == "report_levels") {
        ok = levels(&r->rl, &r->rl_array);
      } else if (key == "transition_levels") {
        ok = levels(&r->tl, &r->tl_array);
      } else if (key == "mode") {
        if (p_ < e_ && *p_ == '"') {
          std::string m;
          ok = string(&m);
          r->mode = (uint8_t)mode_index(m);
        } else {
          r->mode = 0;
          ok = skip(1);
        }
      } else {
        int k = 0;
        while (k < OV_COUNT && key != kOverrideNames[k]) ++k;
        if (k < OV_COUNT && is_number_start()) {
          int64_t i;
          bool ii;
          ok = number(&r->ov[k], &i, &ii);
          if (ii && k == OV_MAX_CANDIDATES) r->ov[k] = (double)i;
          r->ov_mask |= 1u << k;
        } else {
          if (k < OV_COUNT) r->ov_mask &= ~(1u << k);
          ok = skip(1);
        }
      }
      if (!ok) return false;
      ws();
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        continue;
      }
      if (p_ < e_ && *p_ == '}') {
        ++p_;
        return true;
      }
      return fail("Expecting ',' delimiter");
    }
  }
};

// repr(float) as Python 2.7/3 print it inside json.dumps
inline void put_repr(std::string& o, double v) {
  if (std::isnan(v)) {
    o += "NaN";
    return;
  }
  if (std::isinf(v)) {
    o += v > 0 ? "Infinity" : "-Infinity";
    return;
  }
  char buf[40];
  auto r = std::to_chars(buf, buf + sizeof buf, v, std::chars_format::scientific);  // shortest round trip
  const char* s = buf;
  const char* end = r.ptr;
  bool neg = false;
  if (*s == '-') {
    neg = true;
    ++s;
  }
  char dig[24];
  int nd = 0;
  const char* q = s;
  for (; q < end && *q != 'e'; ++q)
    if (*q != '.') dig[nd++] = *q;
  int x = 0;
  std::from_chars(q + 1 + (q[1] == '+'), end, x);
  while (nd > 1 && dig[nd - 1] == '0') --nd;
  if (neg) o.push_back('-');
  if (x >= -4 && x < 16) {
    if (x >= 0) {
      for (int k = 0; k <= x; ++k) o.push_back(k < nd ? dig[k] : '0');
      o.push_back('.');
      if (nd > x + 1) o.append(dig + x + 1, dig + nd);
      else o.push_back('0');
    } else {
      o += "0.";
      for (int k = 0; k < -x - 1; ++k) o.push_back('0');
      o.append(dig, dig + nd);
    }
  } else {
    o.push_back(dig[0]);
    if (nd > 1) {
      o.push_back('.');
      o.append(dig + 1, dig + nd);
    }
    o.push_back('e');
    o.push_back(x < 0 ? '-' : '+');
    const int ax = x < 0 ? -x : x;
    if (ax < 10) o.push_back('0');
    o += std::to_string(ax);
  }
}

}  // namespace otrreq
