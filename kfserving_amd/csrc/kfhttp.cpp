// The model server's HTTP/1.1 front end (include/kfhttp.h).
//
// IO threads each own an epoll set holding the shared listening socket
// (EPOLLEXCLUSIVE: one thread takes each connection, across the pre-forked
// worker processes too), their connections (edge-triggered) and an eventfd on
// which responses for their connections arrive: the native batcher's
// completions (kb_set_done_callback, on a model thread) and the Python
// application's answers (kh_respond).  A connection handles one request at a
// time, in order, as the Python server does (kfserver.py _serve_conn):
// requests pipelined behind it wait in its read buffer.
//
// The parser follows the Python server's (kfserver.py _read_request): the
// request line split on single spaces into exactly three parts, header lines
// partitioned at the first ':' with keys lower-cased and both sides stripped
// (a later duplicate wins), a Content-Length or a chunked body, lines of at
// most 2^20 bytes (asyncio's reader limit); a malformed request gets the 400
// page, a body over max_body_bytes the 413 page, and the connection closes.
#include "kfhttp.h"

#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "kfbatch.h"
#include "kfserve.h"

namespace {

constexpr size_t kMaxLine = 1u << 20;       // asyncio StreamReader limit (start_server)
// read backpressure: while a connection's request is being
// answered, at most this many unparsed bytes are buffered behind it (the
// asyncio server stops reading past 2 x its 2^20 StreamReader limit); the read
// resumes once the answer is out
constexpr size_t kMaxPipelined = size_t(2) << 20;
// bytes one wake-up reads from a connection before the IO thread serves the
// others (edge-triggered: the connection is revisited after this epoll round)
constexpr size_t kReadBudget = size_t(4) << 20;
constexpr uint64_t kListen = ~0ULL, kWake = ~0ULL - 1;
constexpr int kThreadShift = 48;            // tag / id: thread index above the connection id

struct RouteCtx;

struct Route {
  void* batcher = nullptr;
  RouteCtx* ctx = nullptr;
  int n_cols = 0, out_width = 0, out_elem = 0, transform = 0;
  // class labels (kh_add_v1_predict): the prediction is an index into them,
  // each already rendered as json.dumps renders it
  std::shared_ptr<const std::vector<std::string>> labels;
  // lgbserver routes (kh_add_v1_inputs_predict): bodies are {"inputs": ...},
  // columns by these names (back to back, offsets n_cols + 1)
  std::shared_ptr<const std::string> names;
  std::shared_ptr<const std::vector<int32_t>> name_offsets;
  bool v2 = false;   // V2 tensor requests (kh_add_v2_tensor_predict)
};

// where an incomplete chunked body stopped (offsets relative to the request's
// first byte, which stays at Conn::in_off until the request completes), so the
// next read resumes at the chunk it was in instead of re-parsing them all
struct ChunkState {
  bool active = false;
  size_t next = 0;                                  // the next chunk-size line
  int64_t total = 0;
  std::vector<std::pair<size_t, size_t>> spans;     // (offset, size) of the chunks so far
  std::string method, target, version, headers;
  std::unordered_map<std::string, std::string> h;
};

struct Conn {
  uint64_t id = 0;
  int fd = -1;
  std::string in;
  size_t in_off = 0;
  std::string out;
  size_t out_off = 0;
  bool busy = false;         // a request is being answered
  bool peer_gone = false;    // the peer closed while busy: free on the answer
  bool close_after = false;  // close once `out` is written
  bool want_out = false;     // EPOLLOUT armed
  bool peer_eof = false;     // the peer shut its side: answer what is complete, then close
  bool read_paused = false;  // busy with kMaxPipelined bytes behind: resumed by on_done
  ChunkState chunk;
  // the fast-path request in flight
  Route route;
  std::vector<unsigned char> res;
  int64_t rows = 0;
  bool keep = true;
  std::string model, v2_id;   // a V2 tensor answer: the model's name, the request's id text
  bool v2_binary = false;     // ... asked as binary tensor data (binary_data_output)
  // the request handed to Python (kept until kh_respond)
  std::string method, target, version, headers, body;
};

struct Done {
  uint64_t conn = 0;
  bool from_python = false;
  kb_completion c{};
  std::string bytes;   // Python's response; or the model's error text (failed batch)
  bool close_after = false;
};

struct Server;

struct IoThread {
  Server* srv = nullptr;
  int idx = 0;
  int ep = -1, wake = -1;
  std::thread th;
  std::mutex mu;                 // done, new_fds
  std::deque<Done> done;
  std::vector<int> new_fds;      // connections another thread accepted for this one
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> conns;   // this thread only
  uint64_t next_id = 1;
  std::vector<uint64_t> again;   // connections that used their read budget: read on
};

struct Pending {
  uint64_t id;
  Conn* c;
};

struct RouteCtx {   // the done callback's context: its server and batcher
  Server* s = nullptr;
  void* batcher = nullptr;
  std::atomic<int64_t> inflight{0};   // requests submitted through it, not yet completed
};

struct Server {
  kh_config cfg{};
  std::vector<std::unique_ptr<IoThread>> io;
  std::mutex rmu;
  std::unordered_map<std::string, Route> routes;
  std::mutex fmu;
  std::deque<Pending> fq;        // requests for Python
  std::unordered_map<uint64_t, Conn*> handed;   // id -> connection, until kh_respond
  int ffd = -1;
  std::atomic<bool> stop{false};
  std::atomic<int64_t> n_conn{0}, n_native{0}, n_python{0}, n_bad{0};
  std::deque<RouteCtx> ctxs;          // stable addresses, freed with the server
  std::atomic<uint64_t> next_thread{0};   // round robin of accepted connections
  bool started = false;
  int parse_threads = 8;                  // KF_PARSE_THREADS, as fastjson.PARSE_THREADS
};

void signal_fd(int fd) {
  const uint64_t one = 1;
  ssize_t r;
  do {
    r = write(fd, &one, sizeof one);
  } while (r < 0 && errno == EINTR);
}

void drain_fd(int fd) {
  uint64_t v;
  while (read(fd, &v, sizeof v) > 0) {
  }
}

// ------------------------------------------------------------- formatting
// Python's float repr ('r' format, kfserver._json_body -> json.dumps): the
// shortest round-trip digits, fixed notation when the decimal exponent is in
// [-4, 16), else d[.ddd]e[+-]XX.
int repr_double(double v, char* buf, int cap) {
  char s[48];   // the longest: "-d.ddddddddddddddddde-308"
  int n = 0;
  auto put = [&](const char* t) {
    while (*t) s[n++] = *t++;
  };
  if (std::isnan(v)) {
    put("NaN");
  } else if (std::isinf(v)) {
    put(v > 0 ? "Infinity" : "-Infinity");
  } else if (v == 0.0) {
    put(std::signbit(v) ? "-0.0" : "0.0");
  } else {
    // shortest round-trip digits in scientific form: [-]d[.ddd]e[+-]x
    char t[40];
    const auto r = std::to_chars(t, t + sizeof t - 1, v, std::chars_format::scientific);
    *r.ptr = '\0';   // to_chars does not terminate: atoi below reads the exponent
    const char* p = t;
    const char* end = r.ptr;
    if (*p == '-') {
      s[n++] = '-';
      ++p;
    }
    char digits[24] = {};
    int nd = 0;
    while (p < end && *p != 'e') {
      if (*p != '.') digits[nd++] = *p;
      ++p;
    }
    const int exp10 = std::atoi(p + 1);
    const int decpt = exp10 + 1;
    if (decpt <= -4 || decpt > 16) {
      s[n++] = digits[0];
      if (nd > 1) {
        s[n++] = '.';
        for (int k = 1; k < nd; ++k) s[n++] = digits[k];
      }
      s[n++] = 'e';
      s[n++] = exp10 < 0 ? '-' : '+';
      const int a = std::abs(exp10);
      if (a >= 100) s[n++] = static_cast<char>('0' + a / 100);
      s[n++] = static_cast<char>('0' + (a / 10) % 10);
      s[n++] = static_cast<char>('0' + a % 10);
    } else if (decpt <= 0) {
      s[n++] = '0';
      s[n++] = '.';
      for (int k = 0; k < -decpt; ++k) s[n++] = '0';
      for (int k = 0; k < nd; ++k) s[n++] = digits[k];
    } else if (decpt >= nd) {
      for (int k = 0; k < nd; ++k) s[n++] = digits[k];
      for (int k = nd; k < decpt; ++k) s[n++] = '0';
      s[n++] = '.';
      s[n++] = '0';
    } else {
      for (int k = 0; k < decpt; ++k) s[n++] = digits[k];
      s[n++] = '.';
      for (int k = decpt; k < nd; ++k) s[n++] = digits[k];
    }
  }
  if (n >= cap) return -1;
  std::memcpy(buf, s, static_cast<size_t>(n));
  buf[n] = '\0';
  return n;
}

void append_double(std::string& o, double v) {
  char b[48];
  const int n = repr_double(v, b, sizeof b);
  o.append(b, static_cast<size_t>(n));
}

// json.dumps(str) with ensure_ascii (the default): \" \\ \n \r \t \b \f, other
// controls and every non-ASCII code point as \uXXXX (UTF-16 pairs above the
// BMP); invalid UTF-8 reads as U+FFFD, as bytes.decode(errors="replace")
void append_json_string(std::string& o, const std::string& s) {
  o += '"';
  auto u = [&](unsigned cp) {
    char b[8];
    std::snprintf(b, sizeof b, "\\u%04x", cp);
    o += b;
  };
  for (size_t i = 0; i < s.size();) {
    unsigned char ch = static_cast<unsigned char>(s[i]);
    if (ch < 0x80) {
      switch (ch) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        default:
          if (ch < 0x20) u(ch); else o += static_cast<char>(ch);
      }
      ++i;
      continue;
    }
    int n = ch >= 0xF0 ? 3 : ch >= 0xE0 ? 2 : ch >= 0xC0 ? 1 : -1;
    unsigned cp = n == 3 ? ch & 7u : n == 2 ? ch & 15u : ch & 31u;
    bool ok = n > 0 && i + static_cast<size_t>(n) < s.size() + 0;
    for (int k = 1; ok && k <= n; ++k) {
      if (i + static_cast<size_t>(k) >= s.size()) { ok = false; break; }
      const unsigned char cc = static_cast<unsigned char>(s[i + static_cast<size_t>(k)]);
      if ((cc & 0xC0) != 0x80) { ok = false; break; }
      cp = (cp << 6) | (cc & 63u);
    }
    if (!ok || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) {
      u(0xFFFD);
      ++i;
      continue;
    }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u(0xD800 + (cp >> 10));
      u(0xDC00 + (cp & 0x3FF));
    } else {
      u(cp);
    }
    i += static_cast<size_t>(n) + 1;
  }
  o += '"';
}

// kfserver._serialize: status line, the handler's headers, Content-Length,
// Server, and Connection: close when the connection ends
void append_response(std::string& o, int code, const char* reason, const char* ctype,
                     const std::string& body, bool keep, const std::string& extra = std::string()) {
  o += "HTTP/1.1 ";
  o += std::to_string(code);
  o += ' ';
  o += reason;
  o += "\r\nContent-Type: ";
  o += ctype;
  o += extra;   // the handler's further headers, "\r\nName: value" each
  o += "\r\nContent-Length: ";
  o += std::to_string(body.size());
  o += "\r\nServer: kfserving-amd\r\n";
  if (!keep) o += "Connection: close\r\n";
  o += "\r\n";
  o += body;
}

// kfserver.error_response (tornado's error page)
void append_error(std::string& o, int code, const char* reason) {
  const std::string page = "<html><title>" + std::to_string(code) + ": " + reason +
                           "</title><body>" + std::to_string(code) + ": " + reason +
                           "</body></html>";
  append_response(o, code, reason, "text/html; charset=UTF-8", page, false);
}

// ------------------------------------------------------------------- IO
void close_conn(IoThread& t, Conn* c) {
  if (c->fd >= 0) {
    epoll_ctl(t.ep, EPOLL_CTL_DEL, c->fd, nullptr);
    close(c->fd);
    c->fd = -1;
  }
  if (c->busy) {   // an answer is still coming: free it then
    c->peer_gone = true;
    return;
  }
  t.conns.erase(c->id);
}

void arm_out(IoThread& t, Conn* c, bool on) {
  if (c->want_out == on || c->fd < 0) return;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | EPOLLET | (on ? EPOLLOUT : 0u);
  ev.data.u64 = c->id;
  epoll_ctl(t.ep, EPOLL_CTL_MOD, c->fd, &ev);
  c->want_out = on;
}

// write what is pending; false if the connection was closed
bool flush_out(IoThread& t, Conn* c) {
  while (c->out_off < c->out.size()) {
    const ssize_t n = send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off,
                           MSG_NOSIGNAL);
    if (n > 0) {
      c->out_off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      arm_out(t, c, true);
      return true;
    }
    close_conn(t, c);
    return false;
  }
  c->out.clear();
  c->out_off = 0;
  arm_out(t, c, false);
  if (c->close_after) {
    shutdown(c->fd, SHUT_WR);
    close_conn(t, c);
    return false;
  }
  return true;
}

// one line of the read buffer from `pos` (through '\n'): the line without it,
// or npos-style failure: 0 = incomplete, -1 = too long
int take_line(const std::string& in, size_t& pos, std::string& line) {
  const size_t nl = in.find('\n', pos);
  if (nl == std::string::npos) return in.size() - pos > kMaxLine ? -1 : 0;
  if (nl + 1 - pos > kMaxLine) return -1;
  line.assign(in, pos, nl + 1 - pos);
  pos = nl + 1;
  return 1;
}

std::string strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace(static_cast<unsigned char>(s[a]))) ++a;
  while (b > a && std::isspace(static_cast<unsigned char>(s[b - 1]))) --b;
  return s.substr(a, b - a);
}

std::string lower(std::string s) {
  for (char& ch : s) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return s;
}

// int(text) as Python parses a Content-Length / chunk size: optional sign,
// digits (base 10 or 16), surrounding whitespace; false if it would raise
bool py_int(const std::string& t, int base, int64_t* v) {
  const std::string s = strip(t);
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  int64_t x = 0;
  for (; i < s.size(); ++i) {
    const char ch = s[i];
    int d;
    if (ch >= '0' && ch <= '9') d = ch - '0';
    else if (base == 16 && ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
    else if (base == 16 && ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
    else if (ch == '_' && i > 0 && i + 1 < s.size()) continue;
    else return false;
    if (x > (INT64_MAX - d) / base) x = INT64_MAX;   // saturate: far beyond any limit
    else x = x * base + d;
  }
  *v = neg ? -x : x;
  return true;
}

enum class Parse { kIncomplete, kDone, kBad, kTooLarge };

struct Req {
  std::string method, target, version, headers;   // headers: "k: v\n" lines
  std::unordered_map<std::string, std::string> h;
  std::string body;
  size_t end = 0;    // bytes of the read buffer it used
  size_t need = 0;   // kIncomplete with a Content-Length: the request's whole size
};

Parse parse_request(const std::string& in, size_t start, int64_t max_body, Req* r,
                    ChunkState* cs) {
  size_t pos = start;
  std::string line;
  int k;
  if (cs && cs->active) {   // a chunked body part-way: the head and the chunks so far
    r->method = cs->method;
    r->target = cs->target;
    r->version = cs->version;
    r->headers = cs->headers;
    r->h = cs->h;
    pos = start + cs->next;
    goto chunks;
  }
  k = take_line(in, pos, line);
  if (k == 0) return Parse::kIncomplete;
  if (k < 0) return Parse::kBad;
  {
    std::string l = line;
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    size_t a = l.find(' ');
    if (a == std::string::npos) return Parse::kBad;
    size_t b = l.find(' ', a + 1);
    if (b == std::string::npos || l.find(' ', b + 1) != std::string::npos) return Parse::kBad;
    r->method = l.substr(0, a);
    r->target = l.substr(a + 1, b - a - 1);
    r->version = l.substr(b + 1);
  }
  r->headers.clear();
  r->h.clear();
  for (;;) {
    k = take_line(in, pos, line);
    if (k == 0) return Parse::kIncomplete;
    if (k < 0) return Parse::kBad;
    if (line == "\r\n" || line == "\n") break;
    const size_t c = line.find(':');
    const std::string key = lower(strip(c == std::string::npos ? line : line.substr(0, c)));
    const std::string val = c == std::string::npos ? std::string() : strip(line.substr(c + 1));
    r->h[key] = val;
    r->headers += key;
    r->headers += ": ";
    r->headers += val;
    r->headers += '\n';
  }
  {
    auto te = r->h.find("transfer-encoding");
    if (te == r->h.end() || lower(te->second) != "chunked") goto plain;
  }
chunks : {
    // the chunks' spans first; the body is copied only once it is all here.
    // An incomplete body saves where it stopped (ChunkState): the next read
    // resumes at the chunk it was in, so a body of many small chunks costs
    // O(chunks) over all its reads, not per read
    r->body.clear();
    ChunkState local;
    ChunkState& st = cs ? *cs : local;
    if (!st.active) {
      st.total = 0;
      st.spans.clear();
    }
    auto incomplete = [&](size_t chunk_start) {
      if (cs) {
        if (!st.active) {
          st.method = r->method;
          st.target = r->target;
          st.version = r->version;
          st.headers = r->headers;
          st.h = r->h;
        }
        st.active = true;
        st.next = chunk_start - start;
      }
      return Parse::kIncomplete;
    };
    auto fail = [&](Parse p) {
      st.active = false;
      return p;
    };
    for (;;) {
      const size_t chunk_start = pos;
      k = take_line(in, pos, line);
      if (k == 0) return incomplete(chunk_start);
      if (k < 0) return fail(Parse::kBad);
      std::string sz = line.substr(0, line.find(';'));
      int64_t n = 0;
      if (strip(sz).empty()) n = 0;
      else if (!py_int(sz, 16, &n) || n < 0) return fail(Parse::kBad);
      if (n == 0) {
        k = take_line(in, pos, line);   // the line after the last chunk
        if (k == 0) return incomplete(chunk_start);
        if (k < 0) return fail(Parse::kBad);
        break;
      }
      if (st.total + n > max_body) return fail(Parse::kTooLarge);
      if (in.size() - pos < static_cast<size_t>(n)) return incomplete(chunk_start);
      const size_t data = pos;
      pos += static_cast<size_t>(n);
      k = take_line(in, pos, line);
      if (k == 0) return incomplete(chunk_start);
      if (k < 0) return fail(Parse::kBad);
      st.total += n;   // the chunk is whole: counted once, kept relative to start
      st.spans.emplace_back(data - start, static_cast<size_t>(n));
    }
    r->body.reserve(static_cast<size_t>(st.total));
    for (const auto& sp : st.spans) r->body.append(in, start + sp.first, sp.second);
    st.active = false;
    st.spans.clear();
    r->end = pos;
    return Parse::kDone;
  }
plain : {
    r->body.clear();
    int64_t n = 0;
    auto cl = r->h.find("content-length");
    if (cl != r->h.end() && !cl->second.empty() && !py_int(cl->second, 10, &n)) return Parse::kBad;
    if (n > max_body) return Parse::kTooLarge;
    if (n < 0) return Parse::kBad;
    if (in.size() - pos < static_cast<size_t>(n)) {
      r->need = pos - start + static_cast<size_t>(n);
      return Parse::kIncomplete;
    }
    r->body.assign(in, pos, static_cast<size_t>(n));
    pos += static_cast<size_t>(n);
  }
  r->end = pos;
  return Parse::kDone;
}

// "/v1/models/<name>:predict" or "/v2/models/<name>/infer" (query string
// dropped): the model name, or ""; *v2 tells which
std::string predict_route(const std::string& target, bool* v2) {
  const std::string path = target.substr(0, target.find('?'));
  static const std::string pre1 = "/v1/models/", suf1 = ":predict";
  static const std::string pre2 = "/v2/models/", suf2 = "/infer";
  auto match = [&path](const std::string& pre, const std::string& suf) {
    return path.size() > pre.size() + suf.size() && path.compare(0, pre.size(), pre) == 0 &&
           path.compare(path.size() - suf.size(), suf.size(), suf) == 0;
  };
  size_t a, b;
  if (match(pre1, suf1)) {
    a = pre1.size(), b = suf1.size(), *v2 = false;
  } else if (match(pre2, suf2)) {
    a = pre2.size(), b = suf2.size(), *v2 = true;
  } else {
    return std::string();
  }
  std::string name = path.substr(a, path.size() - a - b);
  for (char ch : name)
    if (!(std::isalnum(static_cast<unsigned char>(ch)) || ch == '_' || ch == '-')) return std::string();
  return name;
}

bool process(IoThread& t, Conn* c);

void hand_to_python(IoThread& t, Conn* c, Req& r, bool keep) {
  Server& s = *t.srv;
  c->method = std::move(r.method);
  c->target = std::move(r.target);
  c->version = std::move(r.version);
  c->headers = std::move(r.headers);
  c->body = std::move(r.body);
  c->keep = keep;
  c->busy = true;
  const uint64_t id = (static_cast<uint64_t>(t.idx) << kThreadShift) | c->id;
  {
    std::lock_guard<std::mutex> lk(s.fmu);
    s.fq.push_back({id, c});
    s.handed[id] = c;
  }
  s.n_python.fetch_add(1);
  signal_fd(s.ffd);
}

// the fast path: true if the request went to the batcher
bool try_native(IoThread& t, Conn* c, Req& r, bool keep) {
  Server& s = *t.srv;
  if (r.method != "POST") return false;
  bool v2 = false;
  const std::string name = predict_route(r.target, &v2);
  if (name.empty()) return false;
  for (const char* h : {"ce-specversion", "ce-source", "ce-type", "ce-id"})
    if (r.h.count(h)) return false;   // binary CloudEvents: the application's path
  // /v2/.../infer answers a v1 body as :predict does (ref kfserver.py:77-78);
  // a V2 tensor request (a "datatype" in the body) takes the model's V2
  // route if it has one, and binary tensor data is the application's
  int64_t head_len = -1;   // the binary tensor extension: the JSON part's bytes
  if (v2) {
    auto ih = r.h.find("inference-header-content-length");
    if (ih != r.h.end()) {
      const std::string& t = ih->second;
      if (t.empty() || t.size() > 12 ||
          !std::all_of(t.begin(), t.end(), [](char ch) { return ch >= '0' && ch <= '9'; }))
        return false;   // the application's int() decides
      head_len = std::stoll(t);
      if (head_len > static_cast<int64_t>(r.body.size())) return false;   // its 400
    }
  }
  const bool tensor = v2 && (head_len >= 0 || r.body.find("\"datatype\"") != std::string::npos);
  Route route;
  {
    // the reservation is taken under the route lock: kh_remove_route erases
    // the route under it and then waits for every reservation, so the batcher
    // cannot be destroyed between this lookup and the submit below
    std::lock_guard<std::mutex> lk(s.rmu);
    auto it = s.routes.find(tensor ? "v2:" + name : name);
    if (it == s.routes.end()) return false;
    route = it->second;
    route.ctx->inflight.fetch_add(1);
  }
  struct Reservation {
    RouteCtx* ctx;
    bool held = true;
    ~Reservation() {
      if (held) ctx->inflight.fetch_sub(1);
    }
  } res{route.ctx};
  // the plugin's input checks, as flags above the element rule: a request
  // they would reject goes to the application, which answers its error
  const int rule = route.transform & 0xFF;
  // the parsed values: a buffer the thread keeps for small requests, one of
  // the request's own above kKeepValues (freed with it)
  constexpr size_t kKeepValues = size_t(1) << 19;
  thread_local std::vector<double> xb_kept;
  std::unique_ptr<double[]> xb_own;   // not value-initialised: the parser writes it
  double* xb = nullptr;
  size_t xb_n = 0;
  auto reserve = [&](size_t n) {
    if (n <= kKeepValues) {
      if (xb_kept.size() < n) xb_kept.resize(n);
      xb = xb_kept.data();
    } else {
      xb_own.reset(new double[n]);
      xb = xb_own.get();
    }
    xb_n = n;
  };
  reserve((r.body.size() + 1) / 2);   // a number takes a byte and a separator
  int64_t rows = 0, cols = 0;
  int32_t x_dtype = 1;   // the rows handed to the batcher: float64 (0: float32)
  int64_t id_off = 0, id_len = 0;
  int32_t bin_out = 0;
  if (tensor) {   // {"inputs": [{"name", "shape", "datatype", "data"}], "id"}
    int32_t dt = -1;
    if (kf_parse_v2_tensor(r.body.data(), static_cast<int64_t>(r.body.size()), head_len, xb,
                           static_cast<int64_t>(xb_n), &rows, &cols, &dt, &id_off, &id_len,
                           &bin_out) != KF_PARSED ||
        cols != route.n_cols)
      return false;   // the application: v2.decode_inputs, or an unbatched predict
    if (dt == 0) {    // np.asarray(data, float32): each value rounded to float32
      float* f = reinterpret_cast<float*>(xb);   // in place, front to back
      for (int64_t i = 0; i < rows * cols; ++i) f[i] = static_cast<float>(xb[i]);
      x_dtype = 0;
    }
  } else if (route.names) {   // lgbserver: {"inputs": [{column: [...]}, ...]}
    const int32_t* offs = route.name_offsets->data();
    int rc = kf_parse_inputs(r.body.data(), static_cast<int64_t>(r.body.size()),
                             route.names->data(), offs, route.n_cols, xb,
                             static_cast<int64_t>(xb_n), &rows);
    if (rc == KF_ERR_SPACE && rows > 0 && rows <= (int64_t(1) << 24)) {   // absent columns
      reserve(static_cast<size_t>(rows) * route.n_cols);                 // are NaN: more
      rc = kf_parse_inputs(r.body.data(), static_cast<int64_t>(r.body.size()),   // values
                           route.names->data(), offs, route.n_cols, xb,   // than text
                           static_cast<int64_t>(xb_n), &rows);
    }
    if (rc != KF_PARSED || rows <= 0) return false;
    cols = route.n_cols;
  } else if (kf_parse_instances_mt(r.body.data(), static_cast<int64_t>(r.body.size()),
                                   xb, static_cast<int64_t>(xb_n), &rows, &cols,
                                   s.parse_threads) != KF_PARSED ||
             rows <= 0 || cols != route.n_cols) {
    // bodies of >= 1 MB on parse_threads threads, as the application's
    // fastjson.parse_instances (KF_PARSE_THREADS)
    return false;
  }
  if (route.transform & (KH_CHECK_F32_FINITE | KH_CHECK_NO_NAN)) {
    const bool fin = route.transform & KH_CHECK_F32_FINITE, nonan = route.transform & KH_CHECK_NO_NAN;
    const float* f = reinterpret_cast<const float*>(xb);
    for (int64_t i = 0; i < rows * cols; ++i) {
      const double v = x_dtype == 0 ? f[i] : xb[static_cast<size_t>(i)];
      if (nonan && std::isnan(v)) return false;
      if (fin && std::isinf(static_cast<float>(v))) return false;
    }
  }
  c->route = route;
  c->rows = rows;
  c->keep = keep;
  if (tensor) {
    c->model = name;
    c->v2_id.assign(r.body, static_cast<size_t>(id_off), static_cast<size_t>(id_len));
    c->v2_binary = bin_out != 0;
  }
  c->res.assign(static_cast<size_t>(rows) * route.out_width * route.out_elem, 0);
  c->busy = true;
  const uint64_t tag = KB_TAG_CALLBACK | (static_cast<uint64_t>(t.idx) << kThreadShift) | c->id;
  if (kb_submit_convert(route.batcher, xb, x_dtype, rows, cols, rule, c->res.data(),
                        tag) != KB_OK) {
    c->busy = false;   // the batcher was retired meanwhile: the application answers
    return false;
  }
  res.held = false;    // native_done releases it with the completion
  s.n_native.fetch_add(1);
  return true;
}

// the Python server's bytes for a batched :predict (NativeModelBatcher.submit
// -> model.postprocess -> _ok -> _json_body)
// kfserver.infer's bytes for a V2 tensor request (v2.encode_response: the
// model's output under "predict" in its own datatype, json.dumps of it), or
// for a failed batch HTTPError(500, "Failed to predict ...") as
// error_response renders it
void answer_v2(Conn* c, const kb_completion& d, const std::string& err) {
  std::string body;
  if (d.status != KB_OK) {
    const std::string reason = "Failed to predict " + err;
    std::string line = reason;
    for (char& ch : line)
      if (ch == '\r' || ch == '\n') ch = ' ';   // status_reason
    body = "<html><title>500: " + reason + "</title><body>500: " + reason + "</body></html>";
    append_response(c->out, 500, line.c_str(), "text/html; charset=UTF-8", body, c->keep);
  } else {
    const int w = c->route.out_width;
    body.reserve(128 + static_cast<size_t>(c->rows) * w * 22);
    body += "{\"model_name\": \"";
    body += c->model;
    body += '"';
    if (!c->v2_id.empty()) {
      body += ", \"id\": ";
      body += c->v2_id;
    }
    body += ", \"outputs\": [{\"name\": \"predict\", \"shape\": [";
    body += std::to_string(c->rows);
    if (w > 1) {
      body += ", ";
      body += std::to_string(w);
    }
    body += c->route.out_elem == 4 ? "], \"datatype\": \"FP32\"" : "], \"datatype\": \"FP64\"";
    const size_t n = static_cast<size_t>(c->rows) * w;
    if (c->v2_binary) {   // the binary tensor extension: JSON head, then the raw output
      const size_t raw = n * static_cast<size_t>(c->route.out_elem);
      body += ", \"parameters\": {\"binary_data_size\": ";
      body += std::to_string(raw);
      body += "}}]}";
      const std::string extra = "\r\nInference-Header-Content-Length: " + std::to_string(body.size());
      body.append(reinterpret_cast<const char*>(c->res.data()), raw);   // little endian
      append_response(c->out, 200, "OK", "application/octet-stream", body, c->keep, extra);
      c->close_after = c->close_after || !c->keep;
      std::vector<unsigned char>().swap(c->res);
      c->model.clear();
      c->v2_id.clear();
      c->v2_binary = false;
      return;
    }
    body += ", \"data\": [";
    for (size_t i = 0; i < n; ++i) {
      if (i) body += ", ";
      double v;
      if (c->route.out_elem == 4) {
        float f;
        std::memcpy(&f, c->res.data() + i * 4, 4);
        v = f;
      } else {
        std::memcpy(&v, c->res.data() + i * 8, 8);
      }
      append_double(body, v);
    }
    body += "]}]}";
    append_response(c->out, 200, "OK", "application/json", body, c->keep);
  }
  c->close_after = c->close_after || !c->keep;
  std::vector<unsigned char>().swap(c->res);
  c->model.clear();
  c->v2_id.clear();
  c->v2_binary = false;
}

void answer_native(Conn* c, const kb_completion& d, const std::string& err) {
  if (c->route.v2) {
    answer_v2(c, d, err);
    return;
  }
  std::string body;
  body.reserve(64 + static_cast<size_t>(c->rows) * c->route.out_width * 22);
  if (d.status == KB_OK) {
    body += "{\"message\": \"\", \"batchId\": \"";
    body += d.batch_id;
    body += "\", \"predictions\": [";
    const int w = c->route.out_width;
    for (int64_t i = 0; i < c->rows; ++i) {
      if (i) body += ", ";
      if (w > 1) body += '[';
      for (int j = 0; j < w; ++j) {
        if (j) body += ", ";
        const size_t at = static_cast<size_t>(i * w + j);
        double v;
        if (c->route.out_elem == 4) {
          float f;
          std::memcpy(&f, c->res.data() + at * 4, 4);
          v = f;
        } else {
          std::memcpy(&v, c->res.data() + at * 8, 8);
        }
        const auto* lab = c->route.labels.get();
        if (lab && v >= 0 && v < static_cast<double>(lab->size()))
          body += (*lab)[static_cast<size_t>(v)];   // classes_.take(index)
        else
          append_double(body, v);
      }
      if (w > 1) body += ']';
    }
    body += "]}";
  } else {
    body += "{\"message\": ";
    append_json_string(body, "Failed to predict " + err);
    body += ", \"batchId\": \"\", \"predictions\": null}";
    size_t p = 0;   // tornado's json_encode: "</" -> "<\/"
    while ((p = body.find("</", p)) != std::string::npos) {
      body.replace(p, 2, "<\\/");
      p += 3;
    }
  }
  append_response(c->out, 200, "OK", "application/json; charset=UTF-8", body, c->keep);
  c->close_after = c->close_after || !c->keep;
  std::vector<unsigned char>().swap(c->res);
}

// parse and dispatch what is buffered; false if the connection was freed
bool process(IoThread& t, Conn* c) {
  Server& s = *t.srv;
  while (!c->busy && c->fd >= 0 && !c->close_after) {
    if (c->in_off >= c->in.size()) {
      c->in.clear();
      c->in_off = 0;
      return true;
    }
    Req r;
    const Parse p = parse_request(c->in, c->in_off, s.cfg.max_body_bytes, &r, &c->chunk);
    if (p == Parse::kIncomplete) {
      if (c->in_off > (1u << 16)) {   // keep the buffer from growing at its front
        c->in.erase(0, c->in_off);
        c->in_off = 0;
      }
      // a large body, once its first MB is here, arrives into room for all of
      // it (no re-copy as the buffer grows)
      if (r.need > (1u << 20) && c->in.size() - c->in_off >= (1u << 20) &&
          c->in.capacity() < c->in_off + r.need)
        c->in.reserve(c->in_off + r.need);
      return true;
    }
    if (p == Parse::kBad || p == Parse::kTooLarge) {
      if (p == Parse::kBad) append_error(c->out, 400, "Bad Request");
      else append_error(c->out, 413, "Request Entity Too Large");
      s.n_bad.fetch_add(1);
      c->close_after = true;
      c->in.clear();
      c->in_off = 0;
      return flush_out(t, c);
    }
    c->in_off = r.end;
    auto ch = r.h.find("connection");
    const bool keep = (ch == r.h.end() || lower(ch->second) != "close") && r.version == "HTTP/1.1";
    if (!try_native(t, c, r, keep)) hand_to_python(t, c, r, keep);
  }
  return true;
}

void on_readable(IoThread& t, Conn* c);

// the peer has shut its side and nothing is in flight: every complete request
// has been dispatched (process stops only at a busy connection, an incomplete
// request or the end of the buffer), so a partial request left is answered
// 400 as the Python server's IncompleteReadError is, then the connection
// closes once its answers are written
void finish_at_eof(IoThread& t, Conn* c) {
  if (!c->peer_eof || c->busy || c->fd < 0) return;
  if (c->in_off < c->in.size() && !c->close_after) {
    append_error(c->out, 400, "Bad Request");
    t.srv->n_bad.fetch_add(1);
  }
  c->in.clear();
  c->in_off = 0;
  c->chunk.active = false;
  c->close_after = true;
  flush_out(t, c);
}

void on_done(IoThread& t, Done& d) {
  auto it = t.conns.find(d.conn);
  if (it == t.conns.end()) return;
  Conn* c = it->second.get();
  if (!c->busy) return;
  if (d.from_python) {
    c->out += d.bytes;
    c->close_after = c->close_after || d.close_after;
    c->method.clear();
    c->target.clear();
    c->headers.clear();
    std::string().swap(c->body);
  } else {
    answer_native(c, d.c, d.bytes);
  }
  c->busy = false;
  if (c->peer_gone) {
    t.conns.erase(it);
    return;
  }
  if (!flush_out(t, c) || !process(t, c) || c->fd < 0) return;
  if (c->read_paused) {   // edge-triggered: the bytes left in the socket raise no new event
    c->read_paused = false;
    on_readable(t, c);
    return;
  }
  finish_at_eof(t, c);
}

void on_readable(IoThread& t, Conn* c) {
  char buf[65536];
  size_t since = 0;   // bytes read since the buffer was last parsed
  size_t got = 0;     // bytes read in this wake-up
  while (!c->peer_eof) {
    // backpressure: a request in flight with kMaxPipelined bytes queued behind
    // it stops the reading until its answer is out (on_done resumes it)
    if (c->busy && c->in.size() - c->in_off >= kMaxPipelined) {
      c->read_paused = true;
      return;
    }
    if (got >= kReadBudget) {   // fairness: the thread's other connections first
      t.again.push_back(c->id);
      break;
    }
    const ssize_t n = read(c->fd, buf, sizeof buf);
    if (n > 0) {
      c->in.append(buf, static_cast<size_t>(n));
      since += static_cast<size_t>(n);
      got += static_cast<size_t>(n);
      // a sender that keeps the socket readable does not grow the buffer
      // unparsed: every MB the framing is checked (a bad line or a body over
      // the limit closes the connection now) and complete requests dispatched
      if (since >= (1u << 20) && !c->busy) {
        since = 0;
        if (!process(t, c)) return;
        if (c->fd < 0 || c->close_after) return;   // closing once the answer is out
      }
      continue;
    }
    if (n < 0 && errno == EINTR) continue;
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    // EOF or error: every complete request is still answered, in order (the
    // Python server reads requests until the stream ends), then it closes
    c->peer_eof = true;
  }
  if (!c->busy && !process(t, c)) return;
  if (c->fd >= 0) finish_at_eof(t, c);
}

// a connection joins thread t: registered in its epoll set, then read
void adopt(IoThread& t, int fd) {
  Server& s = *t.srv;
  auto c = std::make_unique<Conn>();
  c->id = t.next_id++;
  c->fd = fd;
  epoll_event ev{};
  ev.events = EPOLLIN | EPOLLRDHUP | EPOLLET;
  ev.data.u64 = c->id;
  if (epoll_ctl(t.ep, EPOLL_CTL_ADD, fd, &ev) != 0) {
    close(fd);
    return;
  }
  Conn* cp = c.get();
  t.conns.emplace(c->id, std::move(c));
  s.n_conn.fetch_add(1);
  on_readable(t, cp);
}

// One connection per wake-up: with EPOLLEXCLUSIVE the next pending one wakes
// another waiter (another worker process's threads included), so a burst of
// connects spreads over the processes.  Inside this process the connections
// go round robin over the IO threads (the request bodies' JSON parse is the
// per-request cost an IO thread pays).
void accept_one(IoThread& t) {
  Server& s = *t.srv;
  int fd;
  do {
    fd = accept4(s.cfg.listen_fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
  } while (fd < 0 && errno == EINTR);
  if (fd < 0) return;   // EAGAIN: another thread or process took it
  const int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  const size_t to = static_cast<size_t>(s.next_thread.fetch_add(1)) % s.io.size();
  if (to == static_cast<size_t>(t.idx)) {
    adopt(t, fd);
    return;
  }
  IoThread& o = *s.io[to];
  {
    std::lock_guard<std::mutex> lk(o.mu);
    o.new_fds.push_back(fd);
  }
  signal_fd(o.wake);
}

void io_main(IoThread* tp) {
  IoThread& t = *tp;
  Server& s = *t.srv;
  epoll_event evs[256];
  std::deque<Done> local;
  std::vector<int> fds;
  std::vector<uint64_t> again;
  while (!s.stop.load()) {
    const int n = epoll_wait(t.ep, evs, 256, t.again.empty() ? 200 : 0);
    again.swap(t.again);   // read on, after this round's events (kReadBudget)
    for (int i = 0; i < n; ++i) {
      const uint64_t key = evs[i].data.u64;
      if (key == kListen) {
        accept_one(t);
      } else if (key == kWake) {
        drain_fd(t.wake);
        {
          std::lock_guard<std::mutex> lk(t.mu);
          local.swap(t.done);
          fds.swap(t.new_fds);
        }
        for (const int fd : fds) adopt(t, fd);
        fds.clear();
        for (Done& d : local) on_done(t, d);
        local.clear();
      } else {
        auto it = t.conns.find(key);
        if (it == t.conns.end()) continue;
        Conn* c = it->second.get();
        if (evs[i].events & EPOLLOUT) {
          if (!flush_out(t, c)) continue;
          if (!c->busy) process(t, c);
          if (t.conns.find(key) == t.conns.end() || c->fd < 0) continue;
        }
        if (evs[i].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) on_readable(t, c);
      }
    }
    for (const uint64_t key : again) {
      auto it = t.conns.find(key);
      if (it != t.conns.end() && it->second->fd >= 0) on_readable(t, it->second.get());
    }
    again.clear();
  }
}

void native_done(void* ctx, const kb_completion* c) {
  RouteCtx& rc = *static_cast<RouteCtx*>(ctx);
  Server& s = *rc.s;
  const size_t ti = static_cast<size_t>((c->tag & ~KB_TAG_CALLBACK) >> kThreadShift);
  if (ti >= s.io.size()) return;
  IoThread& t = *s.io[ti];
  Done d;
  d.conn = c->tag & ((1ULL << kThreadShift) - 1);
  d.c = *c;
  if (c->status != KB_OK) {   // the text now, while the batcher surely exists
    char m[4096];
    // kb_batch_message takes the message lock, not the completion lock held here
    const int n = kb_batch_message(rc.batcher, c->batch_seq, m, sizeof m);
    d.bytes = n >= 0 ? std::string(m, static_cast<size_t>(n)) : std::string("model call failed");
  }
  {
    std::lock_guard<std::mutex> lk(t.mu);
    t.done.push_back(std::move(d));
  }
  rc.inflight.fetch_sub(1);
  signal_fd(t.wake);
}

// no new requests reach the route's batcher (removed from the table): send
// what it holds to the model and wait for those requests' completions, then
// detach the callback, after which the application may destroy the batcher.
// A completion writes into its connection's buffer, so the callback is never
// detached while one is outstanding: after `timeout_s` (< 0: no limit) the
// route stays attached (its context lives as long as the server, so late
// completions still reach their connections) and false is returned
bool detach(RouteCtx* ctx, double timeout_s) {
  kb_flush(ctx->batcher);
  const auto t0 = std::chrono::steady_clock::now();
  double warned = 0;
  while (ctx->inflight.load() > 0) {
    usleep(50);
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_s >= 0 && el >= timeout_s) {
      fprintf(stderr, "kfhttp: %lld request(s) still on a retired route's batcher after %.0f s; "
              "its callback stays attached\n", static_cast<long long>(ctx->inflight.load()), el);
      return false;
    }
    if (el - warned >= 20) {
      warned = el;
      fprintf(stderr, "kfhttp: waiting for %lld request(s) on a batcher (%.0f s)\n",
              static_cast<long long>(ctx->inflight.load()), el);
    }
  }
  kb_set_done_callback(ctx->batcher, nullptr, nullptr);
  return true;
}

}  // namespace

extern "C" {

int32_t kh_abi_version(void) { return KH_ABI_VERSION; }

int kh_repr_double(double v, char* buf, int32_t cap) {
  if (!buf || cap <= 0) return -1;
  return repr_double(v, buf, cap);
}

int kh_create(const kh_config* cfg, void** out) {
  if (!cfg || !out || cfg->abi_version != KH_ABI_VERSION || cfg->listen_fd < 0 ||
      cfg->io_threads < 1 || cfg->io_threads > 256)
    return -1;
  *out = nullptr;
  auto s = std::make_unique<Server>();
  s->cfg = *cfg;
  if (s->cfg.max_body_bytes <= 0) s->cfg.max_body_bytes = 104857600;
  if (const char* e = std::getenv("KF_PARSE_THREADS"))
    s->parse_threads = std::max(1, std::min(8, std::atoi(e)));
  // a failure part-way closes what was opened (no thread is running yet)
  auto fail_sys = [&s]() {
    for (auto& t : s->io) {
      if (t->ep >= 0) close(t->ep);
      if (t->wake >= 0) close(t->wake);
    }
    if (s->ffd >= 0) close(s->ffd);
    return -3;
  };
  s->ffd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (s->ffd < 0) return fail_sys();
  for (int i = 0; i < cfg->io_threads; ++i) {
    s->io.push_back(std::make_unique<IoThread>());
    IoThread* t = s->io.back().get();
    t->srv = s.get();
    t->idx = i;
    t->ep = epoll_create1(EPOLL_CLOEXEC);
    t->wake = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (t->ep < 0 || t->wake < 0) return fail_sys();
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLEXCLUSIVE;
    ev.data.u64 = kListen;
    if (epoll_ctl(t->ep, EPOLL_CTL_ADD, cfg->listen_fd, &ev) != 0) return fail_sys();
    epoll_event wv{};
    wv.events = EPOLLIN;
    wv.data.u64 = kWake;
    if (epoll_ctl(t->ep, EPOLL_CTL_ADD, t->wake, &wv) != 0) return fail_sys();
  }
  *out = s.release();
  return 0;
}

static int add_route(void* h, const char* model, void* batcher, int32_t n_cols,
                     int32_t out_width, int32_t out_elem_bytes, int32_t transform,
                     const char* labels, const int32_t* label_offsets, int32_t n_labels,
                     const char* names, const int32_t* name_offsets, bool v2 = false) {
  if (!h || !model || !batcher || n_cols <= 0 || out_width <= 0 ||
      (out_elem_bytes != 4 && out_elem_bytes != 8) || n_labels < 0 ||
      (n_labels > 0 && (!labels || !label_offsets || out_width != 1)))
    return -1;
  Server& s = *static_cast<Server*>(h);
  const std::string key = v2 ? "v2:" + std::string(model) : std::string(model);
  RouteCtx* ctx;
  {
    std::lock_guard<std::mutex> lk(s.rmu);
    if (s.routes.count(key)) return -1;   // remove the old route first (kh_remove_route)
    s.ctxs.emplace_back();
    ctx = &s.ctxs.back();
    ctx->s = &s;
    ctx->batcher = batcher;
  }
  if (kb_set_done_callback(batcher, native_done, ctx) != KB_OK) return -1;
  Route r;
  r.batcher = batcher;
  r.ctx = ctx;
  r.n_cols = n_cols;
  r.out_width = out_width;
  r.out_elem = out_elem_bytes;
  r.transform = transform;
  if (n_labels > 0) {
    auto v = std::make_shared<std::vector<std::string>>();
    for (int32_t i = 0; i < n_labels; ++i)
      v->emplace_back(labels + label_offsets[i],
                      static_cast<size_t>(label_offsets[i + 1] - label_offsets[i]));
    r.labels = v;
  }
  if (names) {   // an lgbserver route: column names, in the model's order
    r.names = std::make_shared<const std::string>(names, static_cast<size_t>(name_offsets[n_cols]));
    r.name_offsets = std::make_shared<const std::vector<int32_t>>(name_offsets,
                                                                  name_offsets + n_cols + 1);
  }
  r.v2 = v2;
  std::lock_guard<std::mutex> lk(s.rmu);
  s.routes[key] = r;
  return 0;
}

int kh_add_v1_predict(void* h, const char* model, void* batcher, int32_t n_cols,
                      int32_t out_width, int32_t out_elem_bytes, int32_t transform,
                      const char* labels, const int32_t* label_offsets, int32_t n_labels) {
  return add_route(h, model, batcher, n_cols, out_width, out_elem_bytes, transform, labels,
                   label_offsets, n_labels, nullptr, nullptr);
}

int kh_add_v1_inputs_predict(void* h, const char* model, void* batcher, int32_t n_cols,
                             int32_t out_width, int32_t out_elem_bytes, const char* names,
                             const int32_t* name_offsets) {
  if (!names || !name_offsets) return -1;
  return add_route(h, model, batcher, n_cols, out_width, out_elem_bytes, KB_IN_PLAIN, nullptr,
                   nullptr, 0, names, name_offsets);
}

int kh_add_v2_tensor_predict(void* h, const char* model, void* batcher, int32_t n_cols,
                             int32_t out_width, int32_t out_elem_bytes, int32_t transform) {
  if ((transform & 0xFF) != KB_IN_PLAIN) return -1;   // numpy's cast, nothing else
  return add_route(h, model, batcher, n_cols, out_width, out_elem_bytes, transform, nullptr,
                   nullptr, 0, nullptr, nullptr, true);
}

int kh_remove_route(void* h, const char* model) {
  if (!h || !model) return -1;
  Server& s = *static_cast<Server*>(h);
  RouteCtx* ctx;
  {
    std::lock_guard<std::mutex> lk(s.rmu);
    auto it = s.routes.find(model);
    if (it == s.routes.end()) return -1;
    ctx = it->second.ctx;
    s.routes.erase(it);
  }
  return detach(ctx, 20.0) ? 0 : -2;
}

int kh_start(void* h) {
  if (!h) return -1;
  Server& s = *static_cast<Server*>(h);
  if (s.started) return -1;
  s.started = true;
  for (auto& t : s.io) t->th = std::thread(io_main, t.get());
  return 0;
}

int kh_fallback_fd(void* h) { return h ? static_cast<Server*>(h)->ffd : -1; }

int kh_next_fallback(void* h, kh_request* req) {
  if (!h || !req) return -1;
  Server& s = *static_cast<Server*>(h);
  std::lock_guard<std::mutex> lk(s.fmu);
  if (s.fq.empty()) return 0;
  const Pending p = s.fq.front();
  s.fq.pop_front();
  Conn* c = p.c;
  req->id = p.id;
  req->method = c->method.c_str();
  req->target = c->target.c_str();
  req->version = c->version.c_str();
  req->headers = c->headers.data();
  req->headers_len = static_cast<int64_t>(c->headers.size());
  req->body = c->body.data();
  req->body_len = static_cast<int64_t>(c->body.size());
  req->keep_alive = c->keep ? 1 : 0;
  req->reserved = 0;
  return 1;
}

int kh_respond(void* h, uint64_t id, const void* data, int64_t len, int32_t close_after) {
  if (!h || (!data && len > 0) || len < 0) return -1;
  Server& s = *static_cast<Server*>(h);
  {
    std::lock_guard<std::mutex> lk(s.fmu);
    if (!s.handed.erase(id)) return -1;
  }
  const size_t ti = static_cast<size_t>(id >> kThreadShift);
  if (ti >= s.io.size()) return -1;
  IoThread& t = *s.io[ti];
  Done d;
  d.conn = id & ((1ULL << kThreadShift) - 1);
  d.from_python = true;
  d.bytes.assign(static_cast<const char*>(data), static_cast<size_t>(len));
  d.close_after = close_after != 0;
  {
    std::lock_guard<std::mutex> lk(t.mu);
    t.done.push_back(std::move(d));
  }
  signal_fd(t.wake);
  return 0;
}

int kh_get_stats(void* h, kh_stats* st) {
  if (!h || !st) return -1;
  Server& s = *static_cast<Server*>(h);
  st->connections = s.n_conn.load();
  st->native_requests = s.n_native.load();
  st->python_requests = s.n_python.load();
  st->bad_requests = s.n_bad.load();
  return 0;
}

int kh_destroy(void* h) {
  if (!h) return -1;
  Server* s = static_cast<Server*>(h);
  s->stop.store(true);
  for (auto& t : s->io) signal_fd(t->wake);
  for (auto& t : s->io)
    if (t->th.joinable()) t->th.join();
  // requests still on a batcher write into their connection's buffer: every
  // route is detached (its completions arrive in the stopped threads' queues)
  // before anything is freed, with no time limit (a completion
  // after the connections are freed would write into freed memory)
  std::vector<RouteCtx*> live;
  {
    std::lock_guard<std::mutex> lk(s->rmu);
    for (auto& kv : s->routes) live.push_back(kv.second.ctx);
    s->routes.clear();
  }
  for (RouteCtx* c : live) detach(c, -1.0);
  for (auto& t : s->io) {
    for (const int fd : t->new_fds) close(fd);
    for (auto& kv : t->conns)
      if (kv.second->fd >= 0) close(kv.second->fd);
    t->conns.clear();
    epoll_ctl(t->ep, EPOLL_CTL_DEL, s->cfg.listen_fd, nullptr);
    close(t->ep);
    close(t->wake);
  }
  close(s->ffd);
  delete s;
  return 0;
}

}  // extern "C"
