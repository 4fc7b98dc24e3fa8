// Native query_range fetcher: the brain's batched Prometheus requests over
// keep-alive HTTP/1.1 connections, each answer parsed (keyed split) on the
// thread that received it.
//
// At the production 60-s cadence the brain sends a few hundred batched
// requests per cycle (10k canary jobs x 8 metrics: ~280 `pod=~` unions, ~57 MB
// of matrix JSON; 10k continuous jobs x 4 metrics: ~40-160 `app=~` unions).
// Going through a Python HTTP client costs more than the parse; here a batch
// is one call: `nconn` threads take requests off a shared counter, write the
// pre-rendered request bytes, read the response (Content-Length, chunked or
// read-to-close bodies), and run the keyed parser (promparse.cpp) on the body
// while the other threads are still waiting on the server.  ctypes releases
// the GIL for the call.  Connections are kept in the client between batches.
//
// Per request the batch records the HTTP status, the parse result, and four
// times (wait for the first response byte, receive, parse, and the server's
// own time if it reports one in `X-Fm-Server-Us`), so the fetch span of a
// cycle can be attributed to server, wire and client.
//
// Plain http:// only (an https Prometheus goes through the Python client).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

extern "C" int fm_prom_keyed_count(const char* buf, int64_t len, const char* key, int64_t keylen, int64_t* nseries,
                                   int64_t* npoints);
extern "C" int fm_prom_keyed_fill(const char* buf, int64_t len, const char* key, int64_t keylen, double* times,
                                  float* values, int64_t* offsets, uint64_t* key_hash);

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Client {
  sockaddr_storage addr{};
  socklen_t alen = 0;
  int timeout_ms = 90000;
  std::mutex mu;
  std::vector<int> idle;  // keep-alive sockets between batches

  int take() {
    {
      std::lock_guard<std::mutex> g(mu);
      if (!idle.empty()) {
        int fd = idle.back();
        idle.pop_back();
        return fd;
      }
    }
    return -1;
  }
  void give(int fd) {
    std::lock_guard<std::mutex> g(mu);
    idle.push_back(fd);
  }
  // One pooled socket turned out stale (the server or a proxy dropped its
  // idle connections between cycles): the rest of the pool is from the same
  // idle period, so close it all instead of finding out one request at a time.
  void drop_idle() {
    std::vector<int> v;
    {
      std::lock_guard<std::mutex> g(mu);
      v.swap(idle);
    }
    for (int fd : v) ::close(fd);
  }
  int connect_new() {
    int fd = ::socket(addr.ss_family, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
    ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    if (::connect(fd, (const sockaddr*)&addr, alen) != 0) {
      ::close(fd);
      return -1;
    }
    return fd;
  }
  ~Client() {
    for (int fd : idle) ::close(fd);
  }
};

struct Result {
  int64_t status = 0;  // HTTP status; -1 transport error; -2 malformed HTTP; -3 malformed / failed matrix
  std::string err;
  std::vector<double> t;
  std::vector<float> v;
  std::vector<int64_t> off;
  std::vector<uint64_t> kh;
  double wait_s = 0, recv_s = 0, parse_s = 0, server_s = -1;
  int64_t bytes = 0;
};

struct Batch {
  std::vector<Result> res;
};

bool send_all(int fd, const char* p, int64_t n) {
  while (n > 0) {
    ssize_t w = ::send(fd, p, (size_t)n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w;
    n -= w;
  }
  return true;
}

bool ieq_prefix(const char* a, const char* e, const char* lit) {
  for (; *lit; ++a, ++lit)
    if (a >= e || ((*a | 0x20) != (*lit | 0x20))) return false;
  return true;
}

// One response off `fd` into r (body in `body`).  Returns 0 ok, 1 the peer
// closed (or reset) the connection before sending anything (a stale
// keep-alive socket: retry on a new one), -1 transport error -- a receive
// timeout included: a server that is slow to answer is not re-sent the
// request --, -2 malformed.  keep = the connection may be reused.
int read_response(int fd, std::string& buf, std::string& body, Result& r, bool& keep, double t_sent) {
  buf.clear();
  body.clear();
  keep = true;
  char tmp[1 << 16];
  size_t hdr_end = std::string::npos;
  bool first = true;
  double t_first = t_sent;
  while (hdr_end == std::string::npos) {
    ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
    if (k < 0 && errno == EINTR) continue;
    if (k == 0) return buf.empty() ? 1 : -2;
    if (k < 0) {
      const bool reset = errno == ECONNRESET || errno == EPIPE || errno == ENOTCONN;
      return buf.empty() && reset ? 1 : -1;
    }
    if (first) {
      t_first = now_s();
      first = false;
    }
    buf.append(tmp, (size_t)k);
    hdr_end = buf.find("\r\n\r\n");
    if (buf.size() > (1u << 20) && hdr_end == std::string::npos) return -2;
  }
  r.wait_s = t_first - t_sent;
  // status line
  const char* p = buf.data();
  const char* he = p + hdr_end;
  if (he - p < 12 || std::memcmp(p, "HTTP/1.", 7) != 0) return -2;
  r.status = std::atoi(p + 9);
  const bool http10 = p[7] == '0';
  if (http10) keep = false;
  int64_t clen = -1;
  bool chunked = false;
  const char* line = (const char*)std::memchr(p, '\n', (size_t)(he - p));
  while (line && line < he) {
    const char* ls = line + 1;
    const char* le = (const char*)std::memchr(ls, '\n', (size_t)(he + 2 - ls));
    if (!le) le = he;
    if (ieq_prefix(ls, le, "content-length:")) {
      clen = std::atoll(ls + 15);
    } else if (ieq_prefix(ls, le, "transfer-encoding:")) {
      for (const char* q = ls + 18; q + 7 <= le; ++q)
        if (ieq_prefix(q, le, "chunked")) chunked = true;
    } else if (ieq_prefix(ls, le, "connection:")) {
      for (const char* q = ls + 11; q + 5 <= le; ++q)
        if (ieq_prefix(q, le, "close")) keep = false;
    } else if (ieq_prefix(ls, le, "x-fm-server-us:")) {
      r.server_s = 1e-6 * (double)std::atoll(ls + 15);
    }
    line = le < he ? le : nullptr;
  }
  size_t pos = hdr_end + 4;
  auto more = [&]() -> int {  // 1 got bytes, 0 closed, -1 error
    for (;;) {
      ssize_t k = ::recv(fd, tmp, sizeof(tmp), 0);
      if (k < 0 && errno == EINTR) continue;
      if (k > 0) {
        buf.append(tmp, (size_t)k);
        return 1;
      }
      return k == 0 ? 0 : -1;
    }
  };
  if (chunked) {
    for (;;) {
      size_t eol;
      while ((eol = buf.find("\r\n", pos)) == std::string::npos) {
        int m = more();
        if (m <= 0) return m == 0 ? -2 : -1;
      }
      char* endp = nullptr;
      const unsigned long long n = std::strtoull(buf.c_str() + pos, &endp, 16);
      if (endp == buf.c_str() + pos) return -2;
      pos = eol + 2;
      if (n == 0) {  // trailers until the empty line
        for (;;) {
          while ((eol = buf.find("\r\n", pos)) == std::string::npos) {
            int m = more();
            if (m <= 0) return m == 0 ? -2 : -1;
          }
          if (eol == pos) {
            pos = eol + 2;
            break;
          }
          pos = eol + 2;
        }
        break;
      }
      while (buf.size() < pos + n + 2) {
        int m = more();
        if (m <= 0) return m == 0 ? -2 : -1;
      }
      body.append(buf, pos, (size_t)n);
      pos += n + 2;
      if (pos > (1u << 22)) {  // keep the raw buffer small: drop what is decoded
        buf.erase(0, pos);
        pos = 0;
      }
    }
  } else if (clen >= 0) {
    while ((int64_t)(buf.size() - pos) < clen) {
      int m = more();
      if (m <= 0) return m == 0 ? -2 : -1;
    }
    body.assign(buf, pos, (size_t)clen);
  } else {  // read to close
    keep = false;
    for (;;) {
      int m = more();
      if (m < 0) return -1;
      if (m == 0) break;
    }
    body.assign(buf, pos, std::string::npos);
  }
  r.recv_s = now_s() - t_first;
  r.bytes = (int64_t)body.size();
  return 0;
}

void parse_body(const std::string& body, const char* key, int64_t keylen, Result& r) {
  const double t0 = now_s();
  if (r.status != 200) {
    r.err = body.substr(0, 400);
    return;
  }
  int64_t ns = 0, np = 0;
  int rc = fm_prom_keyed_count(body.data(), (int64_t)body.size(), key, keylen, &ns, &np);
  if (rc != 0) {
    r.status = -3;
    r.err = rc == 1 ? "prometheus error: " + body.substr(0, 300) : std::string("malformed prometheus response");
    return;
  }
  r.t.resize((size_t)np);
  r.v.resize((size_t)np);
  r.off.resize((size_t)ns + 1);
  r.kh.resize((size_t)ns);
  fm_prom_keyed_fill(body.data(), (int64_t)body.size(), key, keylen, r.t.data(), r.v.data(), r.off.data(),
                     r.kh.data());
  r.parse_s = now_s() - t0;
}

// application/x-www-form-urlencoded / query-string encoding of one value:
// unreserved bytes as they are, everything else %XX
void pct_append(std::string& out, const char* s, int64_t n) {
  static const char hex[] = "0123456789ABCDEF";
  for (int64_t i = 0; i < n; ++i) {
    const unsigned char ch = (unsigned char)s[i];
    if ((ch >= 'a' && ch <= 'z') || (ch >= 'A' && ch <= 'Z') || (ch >= '0' && ch <= '9') || ch == '-' || ch == '_' ||
        ch == '.' || ch == '~') {
      out.push_back((char)ch);
    } else {
      out.push_back('%');
      out.push_back(hex[ch >> 4]);
      out.push_back(hex[ch & 15]);
    }
  }
}

void render_request(const char* host, const char* strs, const int64_t* so, int64_t post_over, std::string& req) {
  const char* path = strs + so[0];
  const int64_t plen = so[1] - so[0];
  std::string q;
  q.reserve((size_t)(so[2] - so[1]) * 3 / 2 + 16);
  q.append("query=");
  pct_append(q, strs + so[1], so[2] - so[1]);
  q.append(strs + so[2], (size_t)(so[3] - so[2]));
  req.clear();
  if ((int64_t)q.size() > post_over) {
    req.append("POST ").append(path, (size_t)plen).append(" HTTP/1.1\r\nHost: ").append(host);
    req.append("\r\nContent-Type: application/x-www-form-urlencoded\r\nAccept: application/json\r\nContent-Length: ");
    req.append(std::to_string(q.size())).append("\r\n\r\n").append(q);
  } else {
    req.append("GET ").append(path, (size_t)plen).append("?").append(q);
    req.append(" HTTP/1.1\r\nHost: ").append(host).append("\r\nAccept: application/json\r\n\r\n");
  }
}

}  // namespace

// host: a name or address; port: TCP port.  NULL when the name does not resolve.
FM_API void* fm_http_client_new(const char* host, int port, int timeout_ms) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  char ps[16];
  std::snprintf(ps, sizeof(ps), "%d", port);
  if (::getaddrinfo(host, ps, &hints, &res) != 0 || !res) return nullptr;
  auto* c = new Client();
  std::memcpy(&c->addr, res->ai_addr, res->ai_addrlen);
  c->alen = (socklen_t)res->ai_addrlen;
  c->timeout_ms = timeout_ms > 0 ? timeout_ms : 90000;
  ::freeaddrinfo(res);
  return c;
}

FM_API void fm_http_client_free(void* c) { delete static_cast<Client*>(c); }

// n query_range requests.  Request i is four strings packed in strs at
// soff[4i .. 4i+4]: the target path (e.g. /api/v1/query_range), the PromQL
// query (raw UTF-8: it is percent-encoded here, on the worker threads), the
// rest of the parameters already encoded ("&start=..&end=..&step=.."), and the
// label its answer is split by.  A request whose encoded query is longer than
// post_over goes as a form POST (Prometheus accepts POST /api/v1/query_range).
// Runs on min(nconn, n) threads; returns a batch handle (never NULL).
FM_API void* fm_http_batch(void* client, const char* host_hdr, const char* strs, const int64_t* soff, int64_t n,
                           int64_t post_over, int nconn) {
  auto* c = static_cast<Client*>(client);
  auto* b = new Batch();
  b->res.resize((size_t)n);
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    std::string buf, body, req;
    buf.reserve(1 << 20);
    body.reserve(1 << 20);
    int fd = -1;
    for (int64_t i = next++; i < n; i = next++) {
      Result& r = b->res[(size_t)i];
      int rc = 1;
      bool keep = false;
      for (int attempt = 0; attempt < 2 && rc == 1; ++attempt) {
        bool fresh = false;
        // the retry always opens a new connection: another pooled socket
        // from the same idle period would most likely be stale as well
        if (fd < 0 && attempt == 0) fd = c->take();
        if (fd < 0) {
          fd = c->connect_new();
          fresh = true;
        }
        if (fd < 0) {
          rc = -1;
          r.err = std::string("connect: ") + std::strerror(errno);
          break;
        }
        if (attempt == 0) render_request(host_hdr, strs, soff + 4 * i, post_over, req);
        const double t_sent = now_s();
        if (!send_all(fd, req.data(), (int64_t)req.size())) {
          ::close(fd);
          fd = -1;
          rc = fresh ? -1 : 1;  // a stale keep-alive socket: one retry on a new connection
          if (rc == -1) r.err = std::string("send: ") + std::strerror(errno);
          else c->drop_idle();
          continue;
        }
        rc = read_response(fd, buf, body, r, keep, t_sent);
        const int rerr = errno;
        if (rc != 0) {
          ::close(fd);
          fd = -1;
          if (rc == 1 && fresh) {
            rc = -1;
            r.err = "connection closed by the server";
          } else if (rc == 1) {
            c->drop_idle();
          } else if (rc == -1) {
            r.err = rerr == EAGAIN || rerr == EWOULDBLOCK ? std::string("receive timeout")
                                                          : std::string("recv: ") + std::strerror(rerr);
          }
        }
      }
      if (rc == 1) rc = -1;
      if (rc != 0) {
        r.status = rc;
        if (r.err.empty()) r.err = rc == -2 ? "malformed HTTP response" : std::string("recv: ") + std::strerror(errno);
        continue;
      }
      if (!keep) {
        ::close(fd);
        fd = -1;
      }
      parse_body(body, strs + soff[4 * i + 3], soff[4 * i + 4] - soff[4 * i + 3], r);
    }
    if (fd >= 0) c->give(fd);
  };
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(nconn, n));
  std::vector<std::thread> th;
  for (int k = 1; k < T; ++k) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  return b;
}

// Per request: status, series and point counts, bytes, and timing[4] =
// (wait, receive, parse, server) seconds (server -1 when not reported).
FM_API void fm_http_batch_info(void* bh, int64_t* status, int64_t* nseries, int64_t* npoints, int64_t* bytes,
                               double* timing) {
  auto* b = static_cast<Batch*>(bh);
  for (size_t i = 0; i < b->res.size(); ++i) {
    const Result& r = b->res[i];
    status[i] = r.status;
    nseries[i] = (int64_t)r.kh.size();
    npoints[i] = (int64_t)r.t.size();
    bytes[i] = r.bytes;
    timing[4 * i + 0] = r.wait_s;
    timing[4 * i + 1] = r.recv_s;
    timing[4 * i + 2] = r.parse_s;
    timing[4 * i + 3] = r.server_s;
  }
}

// Request i's error text (for status != 200); returns its full length.
FM_API int64_t fm_http_batch_error(void* bh, int64_t i, char* out, int64_t cap) {
  auto* b = static_cast<Batch*>(bh);
  const std::string& e = b->res[(size_t)i].err;
  if (cap > 0) {
    const size_t k = std::min<size_t>(e.size(), (size_t)cap);
    std::memcpy(out, e.data(), k);
  }
  return (int64_t)e.size();
}

// Every successful answer, concatenated in request order: series offsets are
// global (off has sum(nseries) + 1 entries).
FM_API void fm_http_batch_fill(void* bh, double* t, float* v, int64_t* off, uint64_t* kh) {
  auto* b = static_cast<Batch*>(bh);
  int64_t s = 0, p = 0;
  off[0] = 0;
  for (const Result& r : b->res) {
    const size_t ns = r.kh.size();
    if (!r.t.empty()) {
      std::memcpy(t + p, r.t.data(), r.t.size() * sizeof(double));
      std::memcpy(v + p, r.v.data(), r.v.size() * sizeof(float));
    }
    if (ns) std::memcpy(kh + s, r.kh.data(), ns * sizeof(uint64_t));
    for (size_t j = 0; j < ns; ++j) off[s + (int64_t)j + 1] = p + r.off[j + 1];
    s += (int64_t)ns;
    p += (int64_t)r.t.size();
  }
}

FM_API void fm_http_batch_free(void* bh) { delete static_cast<Batch*>(bh); }
