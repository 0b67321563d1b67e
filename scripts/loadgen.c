// loadgen.c — open-loop HTTP/1.1 load generator for the C5 serving benchmark
// (4096 concurrent clients of 1-64-row v1 :predict
// requests at a fixed aggregate QPS; p50/p99 end-to-end latency).
//
// Arrivals are a Poisson process at --qps; each picks rows ~ U{1..64} and a
// pre-built body with that many rows (--bodies file from
// scripts/bench_serving.py).  A request goes to an idle keep-alive
// connection (--conns of them, all opened up front); when none is idle it
// waits in a FIFO, and its latency still counts from its scheduled arrival,
// so queueing shows up in the tail.  --threads T splits the connections and
// the rate over T threads, each its own epoll loop and Poisson process (the
// sum of independent Poisson processes is one at the total rate), for rates
// one loop cannot drive.
//
// Output: one JSON line with p50/p90/p99/max latency (ms) over the requests
// scheduled after --warmup seconds, completed requests and rows per second.
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#define MAXR 64

typedef struct {
  char* req;      // full HTTP request bytes
  int len;
  int rows;
} Req;

typedef struct {
  int fd;
  int busy;
  int64_t job;    // index of the request in flight
  const Req* r;
  int sent;
  char* buf;
  int cap, have;
} Conn;

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static __thread uint64_t rng_state = 88172645463325252ULL;
static uint64_t xr(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}
static double urand(void) { return (xr() >> 11) * (1.0 / 9007199254740992.0); }

typedef struct {      // one thread's share of the load and its results
  uint64_t seed;
  int nconn;
  double qps, dur, warm, t0;
  const Req* reqs;
  uint32_t nv;
  struct sockaddr_in sa;
  int64_t nj;
  double* sched;
  const Req** which;
  double* lat;
  int* status;
  int opened;
  int64_t errors;
} Share;

static void* run_share(void* arg);

static int cmp_d(const void* a, const void* b) {
  double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

static const char* arg(int argc, char** argv, const char* k, const char* d) {
  for (int i = 1; i + 1 < argc; ++i)
    if (!strcmp(argv[i], k)) return argv[i + 1];
  return d;
}

static void* run_share(void* arg) {
  Share* z = (Share*)arg;
  rng_state = z->seed;
  const double qps = z->qps, dur = z->dur, warm = z->warm;
  const int nconn = z->nconn;
  const uint32_t nv = z->nv;
  const struct sockaddr_in sa = z->sa;
  // schedule
  int64_t njobs = (int64_t)(qps * (dur + warm) * 1.05) + 64;
  double* sched = malloc(sizeof(double) * njobs);
  const Req** which = malloc(sizeof(Req*) * njobs);
  double* lat = malloc(sizeof(double) * njobs);
  int* status = calloc(njobs, sizeof(int));
  double t = 0;
  int64_t nj = 0;
  while (nj < njobs) {
    t += -log(1.0 - urand()) / qps;
    if (t >= dur + warm) break;
    sched[nj] = t;
    int r = 1 + (int)(xr() % MAXR);
    which[nj] = &z->reqs[(r - 1) * nv + (xr() % nv)];
    lat[nj] = -1;
    ++nj;
  }

  int ep = epoll_create1(0);
  Conn* cs = calloc((size_t)nconn, sizeof(Conn));
  int opened = 0;
  for (int i = 0; i < nconn; ++i) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) break;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    if (connect(fd, (struct sockaddr*)&sa, sizeof sa) != 0) { close(fd); break; }
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    cs[i].fd = fd;
    cs[i].cap = 1 << 16;
    cs[i].buf = malloc((size_t)cs[i].cap);
    struct epoll_event ev = {.events = EPOLLIN, .data.u32 = (uint32_t)i};
    epoll_ctl(ep, EPOLL_CTL_ADD, fd, &ev);
    ++opened;
  }
  z->opened = opened;
  if (opened == 0) return NULL;
  int* idle = malloc(sizeof(int) * opened);
  int nidle = 0;
  for (int i = opened - 1; i >= 0; --i) idle[nidle++] = i;
  int64_t* fifo = malloc(sizeof(int64_t) * (size_t)nj);
  int64_t fh = 0, ft = 0;

  const double t0 = z->t0;
  int64_t next = 0, done = 0, errors = 0;
  double end_t = t0 + dur + warm + 30.0;   // drain limit

  struct epoll_event evs[1024];
  for (;;) {
    double tn = now_s();
    while (next < nj && t0 + sched[next] <= tn) fifo[ft++] = next++;
    // dispatch queued requests to idle connections
    while (fh < ft && nidle > 0) {
      int c = idle[--nidle];
      Conn* k = &cs[c];
      k->busy = 1;
      k->job = fifo[fh++];
      k->r = which[k->job];
      k->sent = 0;
      k->have = 0;
      ssize_t w = send(k->fd, k->r->req, (size_t)k->r->len, MSG_NOSIGNAL);
      if (w > 0) k->sent = (int)w;
      if (k->sent < k->r->len) {
        struct epoll_event ev = {.events = EPOLLIN | EPOLLOUT, .data.u32 = (uint32_t)c};
        epoll_ctl(ep, EPOLL_CTL_MOD, k->fd, &ev);
      }
    }
    if (next >= nj && done + errors >= nj) break;
    if (tn > end_t) break;
    int timeout_ms = 1;
    if (next < nj) {
      double dt = t0 + sched[next] - now_s();
      timeout_ms = dt <= 0 ? 0 : (int)(dt * 1000.0);
      if (timeout_ms > 5) timeout_ms = 5;
    }
    int n = epoll_wait(ep, evs, 1024, timeout_ms);
    for (int e = 0; e < n; ++e) {
      int c = (int)evs[e].data.u32;
      Conn* k = &cs[c];
      if ((evs[e].events & EPOLLOUT) && k->busy && k->sent < k->r->len) {
        ssize_t w = send(k->fd, k->r->req + k->sent, (size_t)(k->r->len - k->sent), MSG_NOSIGNAL);
        if (w > 0) k->sent += (int)w;
        if (k->sent >= k->r->len) {
          struct epoll_event ev = {.events = EPOLLIN, .data.u32 = (uint32_t)c};
          epoll_ctl(ep, EPOLL_CTL_MOD, k->fd, &ev);
        }
      }
      if (!(evs[e].events & (EPOLLIN | EPOLLERR | EPOLLHUP))) continue;
      for (;;) {
        if (k->have == k->cap) {
          k->cap *= 2;
          k->buf = realloc(k->buf, (size_t)k->cap);
        }
        ssize_t rd = recv(k->fd, k->buf + k->have, (size_t)(k->cap - k->have), 0);
        if (rd > 0) {
          k->have += (int)rd;
          continue;
        }
        if (rd == 0 || (errno != EAGAIN && errno != EWOULDBLOCK)) {   // peer closed
          if (k->busy) { ++errors; k->busy = 0; }
          epoll_ctl(ep, EPOLL_CTL_DEL, k->fd, NULL);
          close(k->fd);
          k->fd = -1;
        }
        break;
      }
      if (!k->busy || k->fd < 0) continue;
      // complete response?  status line + headers + Content-Length body
      char* he = memmem(k->buf, (size_t)k->have, "\r\n\r\n", 4);
      if (!he) continue;
      int hlen = (int)(he - k->buf) + 4;
      int clen = 0;
      char* cl = memmem(k->buf, (size_t)hlen, "Content-Length:", 15);
      if (!cl) cl = memmem(k->buf, (size_t)hlen, "content-length:", 15);
      if (cl) clen = atoi(cl + 15);
      if (k->have < hlen + clen) continue;
      int code = atoi(k->buf + 9);
      lat[k->job] = now_s() - (t0 + sched[k->job]);
      status[k->job] = code;
      ++done;
      k->busy = 0;
      k->have = 0;
      idle[nidle++] = c;
    }
  }

  z->nj = nj;
  z->sched = sched;
  z->which = which;
  z->lat = lat;
  z->status = status;
  z->errors = errors;
  for (int i = 0; i < opened; ++i)
    if (cs[i].fd >= 0) close(cs[i].fd);
  return NULL;
}

int main(int argc, char** argv) {
  const char* host = arg(argc, argv, "--host", "127.0.0.1");
  int port = atoi(arg(argc, argv, "--port", "8080"));
  const char* path = arg(argc, argv, "--path", "/v1/models/model:predict");
  int nconn = atoi(arg(argc, argv, "--conns", "4096"));
  double qps = atof(arg(argc, argv, "--qps", "10000"));
  double dur = atof(arg(argc, argv, "--duration", "10"));
  double warm = atof(arg(argc, argv, "--warmup", "2"));
  const char* bodies = arg(argc, argv, "--bodies", "bodies.bin");
  // --v2-binary: each body starts with a u32, the length of its JSON head (the
  // V2 binary tensor extension's Inference-Header-Content-Length)
  const int v2bin = atoi(arg(argc, argv, "--v2-binary", "0"));

  struct rlimit rl;
  getrlimit(RLIMIT_NOFILE, &rl);
  rl.rlim_cur = rl.rlim_max;
  setrlimit(RLIMIT_NOFILE, &rl);
  if ((rlim_t)nconn + 64 > rl.rlim_cur) nconn = (int)rl.rlim_cur - 64;

  // bodies file: u32 n_variants, then for rows 1..64, n_variants x (u32 len, bytes)
  FILE* f = fopen(bodies, "rb");
  if (!f) { perror("bodies"); return 2; }
  uint32_t nv;
  if (fread(&nv, 4, 1, f) != 1 || nv == 0) { fprintf(stderr, "bad bodies file\n"); return 2; }
  Req* reqs = calloc((size_t)MAXR * nv, sizeof(Req));
  for (int r = 1; r <= MAXR; ++r)
    for (uint32_t v = 0; v < nv; ++v) {
      uint32_t bl;
      if (fread(&bl, 4, 1, f) != 1) { fprintf(stderr, "short bodies file\n"); return 2; }
      char* body = malloc(bl);
      if (fread(body, 1, bl, f) != bl) { fprintf(stderr, "short bodies file\n"); return 2; }
      Req* q = &reqs[(r - 1) * nv + v];
      char hdr[512];
      const char* b = body;
      int hl;
      if (v2bin) {
        uint32_t head;
        if (bl < 4) { fprintf(stderr, "bad binary body\n"); return 2; }
        memcpy(&head, body, 4);
        b = body + 4;
        bl -= 4;
        hl = snprintf(hdr, sizeof hdr,
                      "POST %s HTTP/1.1\r\nHost: %s:%d\r\nContent-Type: application/octet-stream\r\n"
                      "Inference-Header-Content-Length: %u\r\nContent-Length: %u\r\n\r\n", path,
                      host, port, head, bl);
      } else {
        hl = snprintf(hdr, sizeof hdr,
                      "POST %s HTTP/1.1\r\nHost: %s:%d\r\nContent-Type: application/json\r\n"
                      "Content-Length: %u\r\n\r\n", path, host, port, bl);
      }
      q->req = malloc((size_t)hl + bl);
      memcpy(q->req, hdr, (size_t)hl);
      memcpy(q->req + hl, b, bl);
      q->len = hl + (int)bl;
      q->rows = r;
      free(body);
    }
  fclose(f);

  int nthreads = atoi(arg(argc, argv, "--threads", "1"));
  if (nthreads < 1) nthreads = 1;
  if (nthreads > nconn) nthreads = nconn;
  uint64_t seed0 = (uint64_t)atoll(arg(argc, argv, "--seed", "7"));
  struct sockaddr_in sa;
  memset(&sa, 0, sizeof sa);
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  inet_pton(AF_INET, host, &sa.sin_addr);
  Share* sh = calloc((size_t)nthreads, sizeof(Share));
  pthread_t* th = calloc((size_t)nthreads, sizeof(pthread_t));
  const double t0 = now_s() + 0.05 + 0.0005 * nconn;   // after every connect
  for (int k = 0; k < nthreads; ++k) {
    sh[k].seed = (88172645463325252ULL ^ (seed0 * 0x9E3779B97F4A7C15ULL)) + 0x632BE59BD9B4E019ULL * (uint64_t)k;
    sh[k].nconn = nconn / nthreads + (k < nconn % nthreads);
    sh[k].qps = qps / nthreads;
    sh[k].dur = dur;
    sh[k].warm = warm;
    sh[k].t0 = t0;
    sh[k].reqs = reqs;
    sh[k].nv = nv;
    sh[k].sa = sa;
    pthread_create(&th[k], NULL, run_share, &sh[k]);
  }
  int opened = 0;
  int64_t errors = 0, nj = 0;
  for (int k = 0; k < nthreads; ++k) {
    pthread_join(th[k], NULL);
    opened += sh[k].opened;
    errors += sh[k].errors;
    nj += sh[k].nj;
  }
  if (opened == 0) { fprintf(stderr, "could not connect\n"); return 3; }

  // report requests scheduled after warmup
  double* l = malloc(sizeof(double) * (size_t)(nj + 1));
  int64_t m = 0, non200 = 0, rows = 0, lost = 0;
  double first = -1, last = 0;
  for (int k = 0; k < nthreads; ++k) {
    const Share* z = &sh[k];
    for (int64_t i = 0; i < z->nj; ++i) {
      if (z->sched[i] < warm) continue;
      if (z->lat[i] < 0) { ++lost; continue; }
      if (z->status[i] != 200) ++non200;
      l[m++] = z->lat[i];
      rows += z->which[i]->rows;
      double fin = z->sched[i] + z->lat[i];
      if (first < 0 || z->sched[i] < first) first = z->sched[i];
      if (fin > last) last = fin;
    }
  }
  qsort(l, (size_t)m, sizeof(double), cmp_d);
  double span = last - first > 0 ? last - first : 1;
  printf("{\"offered_qps\": %.1f, \"conns\": %d, \"duration_s\": %.2f, \"warmup_s\": %.2f, "
         "\"requests\": %ld, \"completed\": %ld, \"lost\": %ld, \"non200\": %ld, "
         "\"conn_errors\": %ld, \"p50_ms\": %.3f, \"p90_ms\": %.3f, \"p99_ms\": %.3f, "
         "\"max_ms\": %.3f, \"req_per_s\": %.1f, \"rows_per_s\": %.1f, "
         "\"rows_per_request\": \"U{1..64}\"}\n",
         qps, opened, dur, warm, (long)(m + lost), (long)m, (long)lost, (long)non200,
         (long)errors, m ? l[m / 2] * 1e3 : -1, m ? l[(int64_t)(m * 0.9)] * 1e3 : -1,
         m ? l[(int64_t)(m * 0.99)] * 1e3 : -1, m ? l[m - 1] * 1e3 : -1, m / span, rows / span);
  return 0;
}
