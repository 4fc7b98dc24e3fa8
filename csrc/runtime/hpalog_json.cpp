// hpalogs bodies of one brain cycle (service/store.py, api/models.py
// HPALogBatch): the JSON of HPALog.to_dict for every due HPA job,
//
//   {"job_id": .., "created_at": .., "timestamp": .., "hpalog": {"hpascore": ..,
//    "reason": .., "details": [{"metricType": .., "current": .., "upper": ..,
//    "lower": ..}, ...]}}
//
// with json.dumps' separators and Python's float repr, byte for byte (with
// ensure_ascii off).  With one entry per HPA job per cycle (the
// reference writes an hpalogs document per job per brain pass) a 10k-job
// fleet formats 240k floats a cycle; json.dumps over Python dicts took ~50 us
// per entry, this is ~1 us.  Strings are escaped (quote, backslash, control
// characters); other bytes pass through as UTF-8.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

namespace {

inline char* put_lit(char* o, const char* s) {
  const size_t n = std::strlen(s);
  std::memcpy(o, s, n);
  return o + n;
}

inline char* put_str(char* o, const char* s, int64_t n) {
  static const char* hex = "0123456789abcdef";
  *o++ = '"';
  for (int64_t i = 0; i < n; ++i) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    if (c == '"' || c == '\\') {
      *o++ = '\\';
      *o++ = static_cast<char>(c);
    } else if (c == '\n' || c == '\r' || c == '\t' || c == '\b' || c == '\f') {
      *o++ = '\\';
      *o++ = c == '\n' ? 'n' : c == '\r' ? 'r' : c == '\t' ? 't' : c == '\b' ? 'b' : 'f';
    } else if (c < 0x20) {
      o = put_lit(o, "\\u00");
      *o++ = hex[c >> 4];
      *o++ = hex[c & 15];
    } else {
      *o++ = static_cast<char>(c);
    }
  }
  *o++ = '"';
  return o;
}

// Python's float repr: the shortest round-trip digits, written fixed for
// decimal exponents in [-4, 16) (".0" on integral values) and as d.ddde+XX
// otherwise; non-finite values (callers pass finite ones) as json.dumps spells them
inline char* put_float(char* o, double v) {
  if (std::isnan(v)) return put_lit(o, "NaN");
  if (std::isinf(v)) return put_lit(o, v > 0 ? "Infinity" : "-Infinity");
  char b[40];
  char* e = std::to_chars(b, b + sizeof b, v, std::chars_format::scientific).ptr;
  const char* p = b;
  if (*p == '-') *o++ = *p++;
  char dig[24];
  int nd = 0;
  for (; p < e && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  int ex = 0;
  std::from_chars(p + 1 + (p[1] == '+'), e, ex);
  if (ex >= -4 && ex < 16) {
    if (ex >= 0) {
      for (int i = 0; i <= ex; ++i) *o++ = i < nd ? dig[i] : '0';
      *o++ = '.';
      if (nd > ex + 1) {
        for (int i = ex + 1; i < nd; ++i) *o++ = dig[i];
      } else {
        *o++ = '0';
      }
    } else {
      *o++ = '0';
      *o++ = '.';
      for (int i = 0; i < -ex - 1; ++i) *o++ = '0';
      for (int i = 0; i < nd; ++i) *o++ = dig[i];
    }
  } else {
    *o++ = dig[0];
    if (nd > 1) {
      *o++ = '.';
      for (int i = 1; i < nd; ++i) *o++ = dig[i];
    }
    *o++ = 'e';
    *o++ = ex < 0 ? '-' : '+';
    const int a = ex < 0 ? -ex : ex;
    if (a < 10) *o++ = '0';
    o = std::to_chars(o, o + 4, a).ptr;
  }
  return o;
}

}  // namespace

// Upper bound of the bytes fm_hpalog_json writes (escaping can grow a string
// byte to 6).
FM_API int64_t fm_hpalog_bound(int64_t n, int m, int64_t ids_len, int64_t created_len, const int64_t* reason_off,
                               const int32_t* reason_idx, int64_t aliases_len) {
  int64_t tot = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t r = reason_idx[i];
    tot += 6 * (reason_off[r + 1] - reason_off[r]) + 160 + (int64_t)m * 120;
  }
  return tot + 6 * (ids_len + n * created_len + n * aliases_len);
}

namespace {

struct Args {
  int m;
  const char* ids;
  const int64_t* id_off;
  const char* created;
  int64_t created_len;
  const char* ts;
  int64_t ts_len;
  const int64_t* score;
  const int32_t* reason_idx;
  const char* reasons;
  const int64_t* reason_off;
  const char* aliases;
  const int64_t* alias_off;
  const double *cur, *up, *lo;
};

int64_t entry_bound(const Args& a, int64_t i) {
  const int32_t r = a.reason_idx[i];
  return 6 * (a.id_off[i + 1] - a.id_off[i] + a.created_len + a.reason_off[r + 1] - a.reason_off[r]) + 160 +
         (int64_t)a.m * 120 + 6 * (a.alias_off[a.m] - a.alias_off[0]);
}

// Entries [lo, hi) into ``o``; entry i starts at o + (off[i] - off[lo]) relative offsets written to ``off``.
char* format_range(const Args& a, int64_t lo, int64_t hi, char* o, int64_t* off) {
  char* const o0 = o;
  const int m = a.m;
  for (int64_t i = lo; i < hi; ++i) {
    const int32_t r = a.reason_idx[i];
    off[i] = o - o0;
    o = put_lit(o, "{\"job_id\": ");
    o = put_str(o, a.ids + a.id_off[i], a.id_off[i + 1] - a.id_off[i]);
    if (a.created_len > 0) {
      o = put_lit(o, ", \"created_at\": ");
      o = put_str(o, a.created, a.created_len);
    }
    o = put_lit(o, ", \"timestamp\": ");
    std::memcpy(o, a.ts, static_cast<size_t>(a.ts_len));
    o += a.ts_len;
    o = put_lit(o, ", \"hpalog\": {\"hpascore\": ");
    o = std::to_chars(o, o + 24, a.score[i]).ptr;
    o = put_lit(o, ", \"reason\": ");
    o = put_str(o, a.reasons + a.reason_off[r], a.reason_off[r + 1] - a.reason_off[r]);
    o = put_lit(o, ", \"details\": [");
    for (int k = 0; k < m; ++k) {
      if (k) o = put_lit(o, ", ");
      o = put_lit(o, "{\"metricType\": ");
      o = put_str(o, a.aliases + a.alias_off[k], a.alias_off[k + 1] - a.alias_off[k]);
      o = put_lit(o, ", \"current\": ");
      o = put_float(o, a.cur[i * m + k]);
      o = put_lit(o, ", \"upper\": ");
      o = put_float(o, a.up[i * m + k]);
      o = put_lit(o, ", \"lower\": ");
      o = put_float(o, a.lo[i * m + k]);
      *o++ = '}';
    }
    o = put_lit(o, "]}}");
  }
  return o;
}

}  // namespace

// Entry i: job id ids[id_off[i]:id_off[i+1]], reason reasons[reason_off[r]:..]
// with r = reason_idx[i], score[i], and m details (aliases[alias_off[k]:..],
// cur/up/lo[i*m + k]).  Writes the bodies back to back into ``out``, entry i
// at out[body_off[i]:body_off[i+1]]; returns the bytes written, -1 when
// ``cap`` (at least fm_hpalog_bound) is too small.  Runs on up to
// ``threads`` threads (ctypes releases the GIL).
FM_API int64_t fm_hpalog_json(int64_t n, int m, const char* ids, const int64_t* id_off, const char* created,
                              int64_t created_len, double timestamp, const int64_t* score, const int32_t* reason_idx,
                              const char* reasons, const int64_t* reason_off, const char* aliases,
                              const int64_t* alias_off, const double* cur, const double* up, const double* lo,
                              char* out, int64_t cap, int64_t* body_off, int threads) {
  char ts[40];
  char* te = put_float(ts, timestamp);
  const Args a{m, ids, id_off, created, created_len, ts, te - ts, score, reason_idx, reasons, reason_off,
               aliases, alias_off, cur, up, lo};
  int64_t need = 0;
  for (int64_t i = 0; i < n; ++i) need += entry_bound(a, i);
  if (need > cap) return -1;
  const int nt = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(threads, n / 1024)));
  if (nt == 1) {
    char* e = format_range(a, 0, n, out, body_off);
    body_off[n] = e - out;
    return e - out;
  }
  // each thread formats its chunk at its worst-case start, then the chunks are
  // packed down in order
  std::vector<int64_t> lo_i(nt + 1), start(nt + 1, 0), len(nt, 0);
  for (int t = 0; t <= nt; ++t) lo_i[t] = n * t / nt;
  for (int t = 0; t < nt; ++t) {
    int64_t b = 0;
    for (int64_t i = lo_i[t]; i < lo_i[t + 1]; ++i) b += entry_bound(a, i);
    start[t + 1] = start[t] + b;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&, t] { len[t] = format_range(a, lo_i[t], lo_i[t + 1], out + start[t], body_off) - (out + start[t]); });
  for (auto& th : pool) th.join();
  int64_t o = 0;
  for (int t = 0; t < nt; ++t) {
    if (o != start[t]) std::memmove(out + o, out + start[t], static_cast<size_t>(len[t]));
    for (int64_t i = lo_i[t]; i < lo_i[t + 1]; ++i) body_off[i] += o;
    o += len[t];
  }
  body_off[n] = o;
  return o;
}
