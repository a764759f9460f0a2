// Host build of the ingest number parsers (reporter_amd/csrc/otr_ingest.h) so that the
// CPU tests can compare them with Python's own float() / int() / str() on many inputs.
// TEST INFRASTRUCTURE ONLY: the product parses on the GPU (k_ingest_parse).
#define OTR_POW5_QUAL static
#define OTR_INGEST_PARSE_ONLY
#include "../csrc/otr_ingest.h"

using namespace otr;

extern "C" {
// 0 ok, 1 grammar, 2 undecidable
int pc_float(const char* s, int64_t n, double* out) {
  Dec d;
  if (!parse_dec(reinterpret_cast<const uint8_t*>(s), 0, n, d)) return 1;
  return dec_to_double(d, *out) ? 0 : 2;
}
int pc_py2_str(const char* s, int64_t n, double* out) {
  Dec d;
  double v;
  if (!parse_dec(reinterpret_cast<const uint8_t*>(s), 0, n, d)) return 1;
  if (!dec_to_double(d, v)) return 2;
  return py2_str_roundtrip(d, v, *out) ? 0 : 2;
}
int pc_int(const char* s, int64_t n, int64_t* out, int strict) {
  return parse_int(reinterpret_cast<const uint8_t*>(s), 0, n, *out, strict != 0) ? 0 : 1;
}
int pc_ymdhms(const char* s, int64_t n, int64_t* out) {
  return parse_ymdhms(reinterpret_cast<const uint8_t*>(s), 0, n, *out);
}
uint64_t pc_hash(const char* s, int64_t n) { return uuid_hash(reinterpret_cast<const uint8_t*>(s), 0, n); }
}
