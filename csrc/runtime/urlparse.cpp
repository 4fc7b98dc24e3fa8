// Batched parse of barrelman's query_range URLs (foremast_amd/engine/ingest.py
// parse_range's fast shape), for job intake: a canary job carries 2 x M URLs
// whose pod unions run to a kilobyte each, and a 10k-job restart parses 160k
// of them in its first cycle -- regex + percent-decoding per URL in Python
// was ~30 us each.
//
// Accepted shape (anything else reports "not fast" and the caller falls back
// to the general Python parser, which decides):
//   <base>query_range?query=<enc>&start=<num>&end=<num>&step=<digits>
// with <enc> percent-/plus-decoding to
//   <metric>{namespace="<ns>",<pod|app><=|=~>"<v>"}
// where <ns> and <v> hold no '"' or '\', and for =~ every '|'-separated
// alternative is a non-empty [A-Za-z0-9_-]+ literal.  The decoded query must
// be ASCII (the caller slices the decoded buffer by byte offsets).
//
// Reference: barrelman builds these URLs (metricsquery.go:72-99) through the
// service's URL builder (foremast-service/pkg/prometheus/prometheushelper.go:13-43).
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define FM_API extern "C" __attribute__((visibility("default")))

namespace {

int hexval(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

bool is_word(char c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}

bool starts(const char* p, const char* e, const char* lit) {
  const size_t n = std::strlen(lit);
  return (size_t)(e - p) >= n && std::memcmp(p, lit, n) == 0;
}

// [p, e) is \d+(\.\d+)?  (int_only: \d+)
bool number(const char* p, const char* e, bool int_only, double* out) {
  if (p == e) return false;
  const char* q = p;
  while (q < e && *q >= '0' && *q <= '9') ++q;
  if (q == p) return false;
  if (q < e) {
    if (int_only || *q != '.') return false;
    const char* r = ++q;
    while (q < e && *q >= '0' && *q <= '9') ++q;
    if (q == r || q != e) return false;
  }
  char tmp[64];
  const size_t n = (size_t)(e - p);
  if (n >= sizeof(tmp)) return false;
  std::memcpy(tmp, p, n);
  tmp[n] = 0;
  *out = std::strtod(tmp, nullptr);
  return true;
}

// field layout per URL (int64): see fm_parse_ranges
enum { F_OK, F_BASE_B, F_BASE_E, F_MET_B, F_MET_E, F_NS_B, F_NS_E, F_KEY, F_OP, F_VAL_B, F_VAL_E, F_START, F_END,
       F_STEP, F_N };

bool parse_one(const char* u, const char* ue, char* out, int64_t* o, int64_t cap, int64_t* f) {
  // <base>query_range?query=
  static const char kQR[] = "query_range?query=";
  const char* qr = nullptr;
  for (const char* p = u; p + sizeof(kQR) - 1 <= ue; ++p) {
    if (*p == '?') {
      if (p - u >= 11 && std::memcmp(p - 11, "query_range", 11) == 0 && starts(p + 1, ue, "query=")) qr = p - 11;
      break;                                    // the first '?' ends the base
    }
  }
  if (qr == nullptr) return false;
  f[F_BASE_B] = 0;
  f[F_BASE_E] = (qr - u) + 11;
  const char* q = qr + sizeof(kQR) - 1;
  const char* qe = q;
  while (qe < ue && *qe != '&') ++qe;
  // &start=<num>&end=<num>&step=<digits>  (exactly, in this order)
  const char* p = qe;
  if (!starts(p, ue, "&start=")) return false;
  p += 7;
  const char* s0 = p;
  while (p < ue && *p != '&') ++p;
  double v;
  if (!number(s0, p, false, &v)) return false;
  std::memcpy(&f[F_START], &v, 8);
  if (!starts(p, ue, "&end=")) return false;
  p += 5;
  s0 = p;
  while (p < ue && *p != '&') ++p;
  if (!number(s0, p, false, &v)) return false;
  std::memcpy(&f[F_END], &v, 8);
  if (!starts(p, ue, "&step=")) return false;
  p += 6;
  if (!number(p, ue, true, &v)) return false;
  std::memcpy(&f[F_STEP], &v, 8);
  // decode the query into out[o..]
  const int64_t d0 = *o;
  int64_t k = d0;
  for (const char* c = q; c < qe; ++c) {
    if (k >= cap) return false;
    char ch = *c;
    if (ch == '+') {
      ch = ' ';
    } else if (ch == '%') {
      if (qe - c < 3) return false;
      const int h = hexval(c[1]), l = hexval(c[2]);
      if (h < 0 || l < 0) return false;
      ch = (char)(h * 16 + l);
      c += 2;
    }
    if ((unsigned char)ch >= 0x80) return false;   // ASCII only (byte offsets == char offsets)
    out[k++] = ch;
  }
  const char* d = out + d0;
  const char* de = out + k;
  // <metric>{
  const char* m = d;
  if (m == de || !(is_word(*m) || *m == ':') || (*m >= '0' && *m <= '9')) return false;
  while (m < de && (is_word(*m) || *m == ':')) ++m;
  f[F_MET_B] = d0;
  f[F_MET_E] = d0 + (m - d);
  if (!starts(m, de, "{namespace=\"")) return false;
  const char* ns = m + 12;
  const char* nse = ns;
  while (nse < de && *nse != '"' && *nse != '\\') ++nse;
  if (nse >= de || *nse != '"') return false;
  f[F_NS_B] = d0 + (ns - d);
  f[F_NS_E] = d0 + (nse - d);
  const char* kp = nse + 1;
  if (!starts(kp, de, ",")) return false;
  ++kp;
  if (starts(kp, de, "pod")) f[F_KEY] = 0;
  else if (starts(kp, de, "app")) f[F_KEY] = 1;
  else return false;
  kp += 3;
  if (starts(kp, de, "=~\"")) { f[F_OP] = 1; kp += 3; }
  else if (starts(kp, de, "=\"")) { f[F_OP] = 0; kp += 2; }
  else return false;
  const char* ve = kp;
  while (ve < de && *ve != '"' && *ve != '\\') ++ve;
  if (ve + 2 != de || ve[0] != '"' || ve[1] != '}') return false;
  if (ve == kp) return false;                       // empty value
  if (f[F_OP] == 1) {                               // literal alternatives, none empty
    bool empty = true;
    for (const char* c = kp; c < ve; ++c) {
      if (*c == '|') {
        if (empty) return false;
        empty = true;
      } else if (is_word(*c) || *c == '-') {
        empty = false;
      } else {
        return false;
      }
    }
    if (empty) return false;
  }
  f[F_VAL_B] = d0 + (kp - d);
  f[F_VAL_E] = d0 + (ve - d);
  *o = k;
  return true;
}

}  // namespace

// n URLs in buf (URL i = buf[off[i], off[i+1])) -> fields [n][14] int64:
//   ok, base [b, e) in the URL, then in the decoded buffer `out`: metric [b, e),
//   namespace [b, e), key (0 pod, 1 app), op (0 '=', 1 '=~'), values [b, e);
//   start / end / step as float64 bit patterns.
// `out` needs at most buf's length.  Returns the number of fast-shape URLs.
FM_API int64_t fm_parse_ranges(const char* buf, const int64_t* off, int64_t n, char* out, int64_t cap,
                               int64_t* fields) {
  int64_t o = 0, good = 0;
  for (int64_t i = 0; i < n; ++i) {
    int64_t* f = fields + i * F_N;
    std::memset(f, 0, sizeof(int64_t) * F_N);
    const int64_t o0 = o;
    if (parse_one(buf + off[i], buf + off[i + 1], out, &o, cap, f)) {
      f[F_OK] = 1;
      ++good;
    } else {
      o = o0;
    }
  }
  return good;
}
