// Native responder of the fake Prometheus (foremast_amd/demo/promserver.py):
// the HTTP benches' metric store, so that the brain's ingestion -- not a
// Python server -- is what a fetch span measures.
//
// Same answers as the Python FakePrometheus (its tests pin both against the
// per-job answers of engine/sources.py SyntheticSource):
// * `query_range` over GET or form POST, evaluated at start + k*step up to
//   min(end, now), now read from the bench's mmap'd clock file (8 bytes,
//   float64 unix seconds); each point reads the newest raw sample at or
//   before it (raw samples every `raw_step` seconds);
// * plain vector selectors only, exactly one `pod` / `app` matcher (`=`, or
//   `=~` over an alternation of escaped literals), every other matcher `=`;
//   one series per key value, sorted, labels = __name__ + the equality labels
//   + the key label;
// * SyntheticSource's generator: signal key `<base>|<app>`, noise key
//   `<base>|<pod or app>`, fault key = the series' own selector text
//   (ingest.series_identity), fault factors by substring (fm_fault_mag).
//
// One process, one thread per connection (keep-alive HTTP/1.1); the plan of a
// query (its series, label JSON and per-key generator terms) is built once and
// shared by every connection -- a brain repeats its unions every cycle.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <sys/uio.h>

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

extern "C" void fm_synth_many(int64_t K, int64_t nt, const double* level, const double* ad, const double* aw,
                              const double* sph, const double* cph, const uint32_t* kh, const double* t,
                              const double* swd, const double* cwd, const double* sww, const double* cww,
                              const uint32_t* inner, uint32_t c2, float noise, const double* mag, double fault_after,
                              float* out, int threads);
extern "C" void fm_fault_mag(const char* kbuf, const int64_t* koff, int64_t n, const char* sbuf, const int64_t* soff,
                             int64_t nsub, const double* mags, double* out);
extern "C" int64_t fm_prom_format_bound(int64_t nseries, int64_t npts, int64_t label_bytes);
extern "C" int64_t fm_prom_format(int64_t nseries, const char* labels, const int64_t* loff, double t0, double step,
                                  int64_t npts, const float* values, char* out, int64_t cap);

namespace {

constexpr double kPi = 3.141592653589793;

inline uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
inline uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  return hash_u32((a * 0x9E3779B1u) ^ hash_u32((b * 0x85EBCA77u) ^ hash_u32(c + 0x165667B1u)));
}
inline float u01(uint32_t h) { return ((float)(h >> 8) + 1.0f) * (1.0f / 16777216.0f); }

uint32_t crc32(const std::string& s) {  // zlib.crc32
  static uint32_t table[256];
  static bool init = [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    return true;
  }();
  (void)init;
  uint32_t c = 0xFFFFFFFFu;
  for (unsigned char ch : s) c = table[(c ^ ch) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

struct Config {
  std::string fault_buf;
  std::vector<int64_t> fault_off;
  std::vector<double> fault_mag;
  double fault_after = 0, raw_step = 60, noise = 0.02;
  uint32_t seed = 7;
  const double* clock = nullptr;  // mmap'd; null: no clock (+inf)
};

struct Plan {
  std::string err;  // non-empty: a 400 answer
  int64_t K = 0;
  std::string labels;  // JSON label objects, concatenated
  std::vector<int64_t> loff;
  std::vector<double> level, ad, aw, sph, cph, mag;
  std::vector<uint32_t> kh;
  bool has_mag = false;
};

// ---------------------------------------------------------------- PromQL text
bool is_meta(char c) { return std::strchr("\\.^$|?*+()[]{}", c) != nullptr && c != '\0'; }

// Go-style unquote of a double-quoted PromQL string body (promql.unquote)
bool unquote(const std::string& b, std::string& out) {
  out.clear();
  for (size_t i = 0; i < b.size();) {
    char c = b[i];
    if (c != '\\') {
      out.push_back(c);
      ++i;
      continue;
    }
    if (i + 1 >= b.size()) return false;
    char e = b[i + 1];
    auto put_cp = [&](uint32_t cp) {
      if (cp < 0x80) {
        out.push_back((char)cp);
      } else if (cp < 0x800) {
        out.push_back((char)(0xC0 | (cp >> 6)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
      } else if (cp < 0x10000) {
        out.push_back((char)(0xE0 | (cp >> 12)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
      } else {
        out.push_back((char)(0xF0 | (cp >> 18)));
        out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
        out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
        out.push_back((char)(0x80 | (cp & 0x3F)));
      }
    };
    const char* simple = "abfnrtv\\\"'`";
    const char* mapped = "\a\b\f\n\r\t\v\\\"'`";
    const char* p = std::strchr(simple, e);
    if (p && e) {
      out.push_back(mapped[p - simple]);
      i += 2;
    } else if (e == 'x' || e == 'u' || e == 'U') {
      const size_t w = e == 'x' ? 2 : (e == 'u' ? 4 : 8);
      if (i + 2 + w > b.size()) return false;
      uint32_t cp = 0;
      for (size_t k = 0; k < w; ++k) {
        char h = b[i + 2 + k];
        int d = (h >= '0' && h <= '9') ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10
                                                 : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
        if (d < 0) return false;
        cp = cp * 16 + (uint32_t)d;
      }
      if (e == 'x') out.push_back((char)cp);  // Python chr(<256) then UTF-8: not reached by the brain's text
      else put_cp(cp);
      i += 2 + w;
    } else if (e >= '0' && e <= '7') {
      if (i + 4 > b.size()) return false;
      uint32_t cp = 0;
      for (size_t k = 1; k < 4; ++k) {
        char h = b[i + k];
        if (h < '0' || h > '7') return false;
        cp = cp * 8 + (uint32_t)(h - '0');
      }
      out.push_back((char)cp);
      i += 4;
    } else {
      return false;
    }
  }
  return true;
}

// promql.quote
std::string quote(const std::string& v) {
  std::string o = "\"";
  for (char c : v) {
    switch (c) {
      case '\\': o += "\\\\"; break;
      case '"': o += "\\\""; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default: o.push_back(c);
    }
  }
  return o + "\"";
}

std::string json_str(const std::string& v) {
  std::string o = "\"";
  char buf[8];
  for (unsigned char c : v) {
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c < 0x20) {
      std::snprintf(buf, sizeof(buf), "\\u%04x", c);
      o += buf;
    } else o.push_back((char)c);
  }
  return o + "\"";
}

bool literal_alternatives(const std::string& re, std::vector<std::string>& out) {
  out.clear();
  std::string cur;
  for (size_t i = 0; i < re.size(); ++i) {
    char c = re[i];
    if (c == '\\') {
      if (i + 1 >= re.size() || !is_meta(re[i + 1])) return false;
      cur.push_back(re[++i]);
    } else if (c == '|') {
      out.push_back(cur);
      cur.clear();
    } else if (is_meta(c)) {
      return false;
    } else {
      cur.push_back(c);
    }
  }
  out.push_back(cur);
  return true;
}

inline bool ident0(char c) { return std::isalpha((unsigned char)c) || c == '_'; }
inline bool identc(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

struct Matcher {
  std::string k, op, v;
};

// promql.parse_selector
bool parse_selector(const std::string& q, std::string& metric, std::vector<Matcher>& ms) {
  size_t i = 0, n = q.size();
  auto ws = [&]() { while (i < n && std::isspace((unsigned char)q[i])) ++i; };
  ws();
  if (i >= n || !(ident0(q[i]) || q[i] == ':')) return false;
  size_t s = i;
  while (i < n && (identc(q[i]) || q[i] == ':')) ++i;
  metric = q.substr(s, i - s);
  ws();
  ms.clear();
  if (i == n) return true;
  if (q[i] != '{') return false;
  ++i;
  for (;;) {
    ws();
    if (i < n && q[i] == '}') {
      ++i;
      break;
    }
    if (i >= n || !ident0(q[i])) return false;
    s = i;
    while (i < n && identc(q[i])) ++i;
    Matcher m;
    m.k = q.substr(s, i - s);
    ws();
    if (q.compare(i, 2, "=~") == 0 || q.compare(i, 2, "!=") == 0 || q.compare(i, 2, "!~") == 0) {
      m.op = q.substr(i, 2);
      i += 2;
    } else if (i < n && q[i] == '=') {
      m.op = "=";
      ++i;
    } else {
      return false;
    }
    ws();
    if (i >= n || q[i] != '"') return false;
    s = ++i;
    while (i < n && q[i] != '"') i += (q[i] == '\\') ? 2 : 1;
    if (i >= n) return false;
    if (!unquote(q.substr(s, i - s), m.v)) return false;
    ++i;
    ms.push_back(std::move(m));
    ws();
    if (i < n && q[i] == ',') ++i;
  }
  ws();
  return i == n;
}

std::string replace_all(std::string s, const std::string& from) {
  size_t p;
  while ((p = s.find(from)) != std::string::npos) s.erase(p, from.size());
  return s;
}

std::string app_of_pod(const std::string& pod) {
  std::vector<size_t> dash;
  for (size_t i = 0; i < pod.size(); ++i)
    if (pod[i] == '-') dash.push_back(i);
  if (dash.size() < 2) return pod;
  return pod.substr(0, dash[dash.size() - 2]);
}

std::shared_ptr<Plan> make_plan(const std::string& q, const Config& cfg) {
  auto P = std::make_shared<Plan>();
  std::string metric;
  std::vector<Matcher> ms;
  if (!parse_selector(q, metric, ms)) {
    P->err = "unsupported query";
    return P;
  }
  int kp = -1, nk = 0;
  for (size_t i = 0; i < ms.size(); ++i)
    if ((ms[i].k == "pod" || ms[i].k == "app") && (ms[i].op == "=" || ms[i].op == "=~")) {
      kp = (int)i;
      ++nk;
    }
  bool others_eq = true;
  for (size_t i = 0; i < ms.size(); ++i)
    if ((int)i != kp && ms[i].op != "=") others_eq = false;
  if (nk != 1 || !others_eq) {
    P->err = "fake prometheus: unsupported matchers";
    return P;
  }
  const Matcher& km = ms[(size_t)kp];
  std::vector<std::string> alts;
  if (km.op == "=") {
    alts = {km.v};
  } else if (!literal_alternatives(km.v, alts)) {
    P->err = "fake prometheus: non-literal regex";
    return P;
  }
  std::set<std::string> uniq;
  for (auto& a : alts)
    if (!a.empty()) uniq.insert(a);
  const std::string base = replace_all(replace_all(metric, "namespace_pod_"), "namespace_app_pod_");
  // label JSON: __name__ then the other labels sorted by name (json.dumps of
  // {"__name__": m, **dict(sorted(labels))})
  std::vector<std::pair<std::string, std::string>> lab;
  for (size_t i = 0; i < ms.size(); ++i)
    if ((int)i != kp) lab.push_back({ms[i].k, ms[i].v});
  lab.push_back({km.k, std::string()});
  std::sort(lab.begin(), lab.end(), [](auto& a, auto& b) { return a.first < b.first; });
  // the series identity: the selector with the key matcher pinned (render_query)
  std::vector<std::string> pre_parts;
  P->K = (int64_t)uniq.size();
  std::vector<std::string> fkeys;
  P->loff.push_back(0);
  for (const std::string& v : uniq) {
    std::string L = "{\"__name__\":" + json_str(metric);
    for (auto& kv : lab) L += "," + json_str(kv.first) + ":" + json_str(kv.first == km.k ? v : kv.second);
    L += "}";
    P->labels += L;
    P->loff.push_back((int64_t)P->labels.size());
    std::string id = metric + "{";
    for (size_t i = 0; i < ms.size(); ++i) {
      if (i) id += ",";
      id += ms[i].k + "=" + quote((int)i == kp ? v : ms[i].v);
    }
    id += "}";
    fkeys.push_back(std::move(id));
    const std::string sig = base + "|" + (km.k == "pod" ? app_of_pod(v) : v);
    const std::string noise = base + "|" + v;
    const uint32_t h = crc32(sig) ^ cfg.seed;
    const double u0 = u01(hash3(h, 0, 0x51ED27)), u1 = u01(hash3(h, 1, 0x51ED27)),
                 u2 = u01(hash3(h, 2, 0x51ED27)), u3 = u01(hash3(h, 3, 0x51ED27));
    P->level.push_back(1.0 + 99.0 * u0);
    P->ad.push_back(0.1 + 0.3 * u1);
    P->aw.push_back(0.01 + 0.04 * u2);
    const double ph = 2 * kPi * u3;
    P->sph.push_back(std::sin(ph));
    P->cph.push_back(std::cos(ph));
    P->kh.push_back(crc32(noise) ^ cfg.seed);
  }
  const int64_t nf = (int64_t)cfg.fault_mag.size();
  if (nf && P->K) {
    std::string kb;
    std::vector<int64_t> ko{0};
    for (auto& f : fkeys) {
      kb += f;
      ko.push_back((int64_t)kb.size());
    }
    P->mag.resize((size_t)P->K);
    fm_fault_mag(kb.data(), ko.data(), P->K, cfg.fault_buf.data(), cfg.fault_off.data(), nf, cfg.fault_mag.data(),
                 P->mag.data());
    for (double m : P->mag) P->has_mag |= (m != 1.0);
  }
  return P;
}

bool parse_step(const std::string& s, double& out) {
  char* e = nullptr;
  out = std::strtod(s.c_str(), &e);
  if (e && *e == '\0' && e != s.c_str()) return true;
  double tot = 0;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = i;
    while (j < s.size() && (std::isdigit((unsigned char)s[j]) || s[j] == '.')) ++j;
    if (j == i) return false;
    const double x = std::atof(s.substr(i, j - i).c_str());
    double u;
    if (s.compare(j, 2, "ms") == 0) { u = 1e-3; j += 2; }
    else if (j < s.size() && s[j] == 's') { u = 1; ++j; }
    else if (j < s.size() && s[j] == 'm') { u = 60; ++j; }
    else if (j < s.size() && s[j] == 'h') { u = 3600; ++j; }
    else if (j < s.size() && s[j] == 'd') { u = 86400; ++j; }
    else if (j < s.size() && s[j] == 'w') { u = 604800; ++j; }
    else if (j < s.size() && s[j] == 'y') { u = 31536000; ++j; }
    else return false;
    tot += x * u;
    i = j;
  }
  out = tot;
  return true;
}

std::string pct_decode(const char* s, size_t n) {  // urllib.parse.unquote_plus
  auto hv = [](char h) {
    return (h >= '0' && h <= '9') ? h - '0' : (h >= 'a' && h <= 'f') ? h - 'a' + 10 : (h >= 'A' && h <= 'F') ? h - 'A' + 10 : -1;
  };
  std::string o;
  o.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const char c = s[i];
    if (c == '+') {
      o.push_back(' ');
      continue;
    }
    if (c == '%' && i + 2 < n + 0 + 1 && i + 2 <= n - 1) {
      const int a = hv(s[i + 1]), b = hv(s[i + 2]);
      if (a >= 0 && b >= 0) {
        o.push_back((char)(a * 16 + b));
        i += 2;
        continue;
      }
    }
    o.push_back(c);
  }
  return o;
}

struct Server {
  Config cfg;
  std::mutex mu;
  std::unordered_map<std::string, std::shared_ptr<Plan>> plans;  // by the still-encoded query text

  std::shared_ptr<Plan> plan_of(const std::string& enc) {
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = plans.find(enc);
      if (it != plans.end()) return it->second;
    }
    auto p = make_plan(pct_decode(enc.data(), enc.size()), cfg);
    std::lock_guard<std::mutex> g(mu);
    if (plans.size() > 16384) plans.clear();
    plans[enc] = p;
    return p;
  }

  double now() const { return cfg.clock ? *(volatile const double*)cfg.clock : INFINITY; }

  // (status, body) of one query_range parameter string
  std::pair<int, std::string> answer(const std::string& raw) {
    std::string qenc, ss, es, st = "60";
    bool hq = false, hs = false, he = false;
    size_t i = 0;
    while (i <= raw.size()) {
      size_t j = raw.find('&', i);
      if (j == std::string::npos) j = raw.size();
      const size_t eq = raw.find('=', i);
      if (eq != std::string::npos && eq < j) {
        const std::string k = raw.substr(i, eq - i);
        const char* v = raw.data() + eq + 1;
        const size_t vn = j - eq - 1;
        if (k == "query") { qenc.assign(v, vn); hq = true; }
        else if (k == "start") { ss = pct_decode(v, vn); hs = true; }
        else if (k == "end") { es = pct_decode(v, vn); he = true; }
        else if (k == "step") { st = pct_decode(v, vn); }
      }
      i = j + 1;
    }
    const char* bad = "{\"status\":\"error\",\"errorType\":\"bad_data\",\"error\":\"missing or bad parameters\"}";
    if (!hq || !hs || !he) return {400, bad};
    char* e1 = nullptr;
    char* e2 = nullptr;
    const double start = std::strtod(ss.c_str(), &e1), end = std::strtod(es.c_str(), &e2);
    if (e1 == ss.c_str() || *e1 || e2 == es.c_str() || *e2) return {400, bad};
    double step;
    if (!parse_step(st, step) || !(step > 0))
      return {400, "{\"status\":\"error\",\"errorType\":\"bad_data\",\"error\":\"bad step\"}"};
    auto P = plan_of(qenc);
    if (!P->err.empty())
      return {400, "{\"status\":\"error\",\"errorType\":\"bad_data\",\"error\":" + json_str(P->err) + "}"};
    const double hi = std::min(end, now());
    const int64_t n = hi >= start ? (int64_t)std::floor((hi - start) / step + 1e-9) + 1 : 0;
    std::vector<float> grid((size_t)(P->K * std::max<int64_t>(n, 0)));
    if (n > 0 && P->K > 0) {
      std::vector<double> tr((size_t)n), swd((size_t)n), cwd((size_t)n), sww((size_t)n), cww((size_t)n);
      std::vector<uint32_t> inner((size_t)n);
      const uint32_t hs0 = hash_u32((uint32_t)(0 + 0x165667B1u));
      const uint32_t c2 = hash_u32((uint32_t)(0x68E31DA4ull * 0x85EBCA77ull) ^ hs0);
      for (int64_t k = 0; k < n; ++k) {
        const double tg = start + step * (double)k;
        const double t = std::floor(tg / cfg.raw_step + 1e-9) * cfg.raw_step;
        tr[(size_t)k] = t;
        const double wd = 2 * kPi * t / 86400.0, ww = 2 * kPi * t / 604800.0;
        swd[(size_t)k] = std::sin(wd);
        cwd[(size_t)k] = std::cos(wd);
        sww[(size_t)k] = std::sin(ww);
        cww[(size_t)k] = std::cos(ww);
        const uint32_t ti = (uint32_t)((int64_t)(t / cfg.raw_step) & 0xFFFFFFFF);
        inner[(size_t)k] = hash_u32((ti * 0x85EBCA77u) ^ hs0);
      }
      fm_synth_many(P->K, n, P->level.data(), P->ad.data(), P->aw.data(), P->sph.data(), P->cph.data(), P->kh.data(),
                    tr.data(), swd.data(), cwd.data(), sww.data(), cww.data(), inner.data(), c2, (float)cfg.noise,
                    P->has_mag ? P->mag.data() : nullptr, cfg.fault_after, grid.data(), 1);
    }
    const int64_t cap = fm_prom_format_bound(P->K, std::max<int64_t>(n, 0), (int64_t)P->labels.size());
    std::string body((size_t)cap, '\0');
    const int64_t w = fm_prom_format(P->K, P->labels.data(), P->loff.data(), start, step, std::max<int64_t>(n, 0),
                                     grid.data(), body.data(), cap);
    if (w < 0) return {500, "{\"status\":\"error\",\"error\":\"format\"}"};
    body.resize((size_t)w);
    return {200, std::move(body)};
  }

  void serve_conn(int fd) {
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::string buf;
    char tmp[1 << 16];
    for (;;) {
      size_t he;
      while ((he = buf.find("\r\n\r\n")) == std::string::npos) {
        ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
        if (k <= 0) {
          ::close(fd);
          return;
        }
        buf.append(tmp, (size_t)k);
      }
      const auto t0 = std::chrono::steady_clock::now();
      const size_t le = buf.find("\r\n");
      const std::string line = buf.substr(0, le);
      int64_t clen = 0;
      bool close_after = line.find("HTTP/1.0") != std::string::npos;
      for (size_t p = le + 2; p < he;) {
        size_t q = buf.find("\r\n", p);
        if (q == std::string::npos || q > he) q = he;
        std::string h = buf.substr(p, q - p);
        for (auto& c : h) c = (char)std::tolower((unsigned char)c);
        if (h.rfind("content-length:", 0) == 0) clen = std::atoll(h.c_str() + 15);
        if (h.rfind("connection:", 0) == 0 && h.find("close") != std::string::npos) close_after = true;
        p = q + 2;
      }
      while ((int64_t)(buf.size() - he - 4) < clen) {
        ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
        if (k <= 0) {
          ::close(fd);
          return;
        }
        buf.append(tmp, (size_t)k);
      }
      const std::string body = buf.substr(he + 4, (size_t)clen);
      buf.erase(0, he + 4 + (size_t)clen);
      const size_t sp1 = line.find(' ');
      const size_t sp2 = line.find(' ', sp1 + 1);
      const std::string method = line.substr(0, sp1);
      const std::string target = sp1 == std::string::npos ? "" : line.substr(sp1 + 1, sp2 - sp1 - 1);
      const size_t qm = target.find('?');
      const std::string path = target.substr(0, qm);
      const std::string qs = qm == std::string::npos ? "" : target.substr(qm + 1);
      auto ends = [&](const char* suf) {
        const size_t n = std::strlen(suf);
        return path.size() >= n && path.compare(path.size() - n, n, suf) == 0;
      };
      std::pair<int, std::string> r;
      if (ends("/api/v1/query_range")) {
        std::string raw = qs;
        if (method == "POST" && !body.empty()) raw += (raw.empty() ? "" : "&") + body;
        r = answer(raw);
      } else if (ends("/-/healthy")) {
        r = {200, "ok"};
      } else {
        r = {404, "{\"status\":\"error\",\"error\":\"not found\"}"};
      }
      const long us = (long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0)
                          .count();
      std::string hdr = "HTTP/1.1 " + std::to_string(r.first) + (r.first == 200 ? " OK" : " Error") +
                        "\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(r.second.size()) +
                        "\r\nX-Fm-Server-Us: " + std::to_string(us) + "\r\n" +
                        (close_after ? "Connection: close\r\n" : "") + "\r\n";
      iovec iov[2] = {{hdr.data(), hdr.size()}, {r.second.data(), r.second.size()}};
      msghdr mh{};
      mh.msg_iov = iov;
      mh.msg_iovlen = 2;
      size_t left = hdr.size() + r.second.size();
      while (left > 0) {
        ssize_t w = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
        if (w <= 0) {
          ::close(fd);
          return;
        }
        left -= (size_t)w;
        size_t adv = (size_t)w;
        while (adv > 0 && mh.msg_iovlen > 0) {
          if (adv >= mh.msg_iov[0].iov_len) {
            adv -= mh.msg_iov[0].iov_len;
            ++mh.msg_iov;
            --mh.msg_iovlen;
          } else {
            mh.msg_iov[0].iov_base = (char*)mh.msg_iov[0].iov_base + adv;
            mh.msg_iov[0].iov_len -= adv;
            adv = 0;
          }
        }
      }
      if (close_after) {
        ::close(fd);
        return;
      }
    }
  }
};

}  // namespace

// Serve forever on the listening socket `lfd` (one thread per connection).
// faults: nf substrings packed at fbuf[foff[j], foff[j+1]) with factors mags[j]
// (SyntheticSource.faults, in its order).  clock_path: the bench's 8-byte
// clock file, or NULL/"" for no clock.  Returns only on a setup error (-1).
FM_API int fm_fakeprom_serve(int lfd, const char* clock_path, const char* fbuf, const int64_t* foff, int64_t nf,
                             const double* mags, double fault_after, double raw_step, double noise, uint32_t seed) {
  auto* S = new Server();  // lives for the process
  S->cfg.fault_buf.assign(fbuf ? fbuf : "", nf ? (size_t)foff[nf] : 0);
  S->cfg.fault_off.assign(foff, foff + nf + 1);
  S->cfg.fault_mag.assign(mags, mags + nf);
  S->cfg.fault_after = fault_after;
  S->cfg.raw_step = raw_step;
  S->cfg.noise = noise;
  S->cfg.seed = seed;
  if (clock_path && *clock_path) {
    int cfd = ::open(clock_path, O_RDONLY);
    if (cfd < 0) return -1;
    void* m = ::mmap(nullptr, 8, PROT_READ, MAP_SHARED, cfd, 0);
    ::close(cfd);
    if (m == MAP_FAILED) return -1;
    S->cfg.clock = (const double*)m;
  }
  for (;;) {
    int fd = ::accept(lfd, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      return -1;
    }
    std::thread([S, fd] { S->serve_conn(fd); }).detach();
  }
}
