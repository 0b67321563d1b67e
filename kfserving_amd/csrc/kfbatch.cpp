// The serving path's request batcher in native code (include/kfbatch.h).
//
// Replaces pkg/batcher/handler.go:98-263 (BatchHandler.batch / batchPredict).
// One mutex guards the forming batch and the queue of flushed batches; a
// timer thread flushes the forming batch when MaxLatency has elapsed since its
// first request (a timed wait on CLOCK_MONOTONIC with the thread's timer slack
// at 1 ns, instead of the Go loop's 100 us poll); kb_submit flushes it when a
// request takes it to MaxBatchSize rows.  `max_inflight` model threads take
// flushed batches in order, call the model (ti_predict) on the batch's
// contiguous rows, copy every request's rows of the output into the request's
// own buffer and post one completion per request to a queue signalled through
// an eventfd.
#include "kfbatch.h"

#include <poll.h>
#include <sys/eventfd.h>
#include <sys/prctl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <limits>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

// libstdc++'s steady_clock is CLOCK_MONOTONIC: a deadline in mono_ns() units
std::chrono::steady_clock::time_point steady_at(int64_t ns) {
  return std::chrono::steady_clock::time_point(std::chrono::nanoseconds(ns));
}

struct Waiter {
  uint64_t tag;
  unsigned char* out;
  int64_t lo, hi;   // the request's rows of the batch
};

struct Batch {
  std::vector<unsigned char> x;   // rows x n_cols elements, dense
  int64_t rows = 0;
  int64_t start_ns = 0;           // Start (handler.go:163-165): first request's arrival
  uint64_t seq = 0;
  std::vector<Waiter> waiters;
};

constexpr size_t kMaxMessages = 1024;   // failed batches whose text is kept

struct Batcher {
  kb_config cfg{};
  kb_predict_fn predict = nullptr;
  void* model = nullptr;
  kb_error_fn err = nullptr;
  kb_done_fn done_fn = nullptr;   // completions of KB_TAG_CALLBACK requests
  void* done_ctx = nullptr;
  size_t x_row = 0, o_row = 0;   // bytes per input / output row
  int64_t max_rows = 0, max_latency_ns = 0;
  int efd = -1;

  std::mutex mu;   // forming, ready, seq, stop, spare
  std::condition_variable timer_cv, work_cv;
  Batch forming;
  std::deque<Batch> ready;
  std::vector<std::vector<unsigned char>> spare;   // input buffers to reuse
  uint64_t seq = 0;
  bool stop = false;

  std::mutex cq_mu;
  std::deque<kb_completion> cq;

  std::mutex msg_mu;
  std::unordered_map<uint64_t, std::string> msgs;
  std::deque<uint64_t> msg_order;

  std::mutex st_mu;
  kb_stats st{};
  std::mt19937_64 rng{std::random_device{}()};

  std::thread timer;
  std::vector<std::thread> workers;
};

// forming -> ready (under b.mu).  `full`: flushed by MaxBatchSize.
void flush_locked(Batcher& b, bool full) {
  if (b.forming.rows == 0) return;
  b.forming.seq = ++b.seq;
  {
    std::lock_guard<std::mutex> lk(b.st_mu);
    b.st.batches += 1;
    b.st.rows += b.forming.rows;
    if (b.forming.rows > b.st.max_batch_rows) b.st.max_batch_rows = b.forming.rows;
    if (full) b.st.full_flushes += 1; else b.st.timer_flushes += 1;
  }
  b.ready.push_back(std::move(b.forming));
  b.forming = Batch();
  b.work_cv.notify_one();
}

void timer_main(Batcher* bp) {
  Batcher& b = *bp;
  (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);   // wake at the deadline, not up to 50 us later
  std::unique_lock<std::mutex> lk(b.mu);
  while (!b.stop) {
    if (b.forming.rows == 0) {
      b.timer_cv.wait(lk);
      continue;
    }
    const int64_t deadline = b.forming.start_ns + b.max_latency_ns;
    if (mono_ns() >= deadline) {   // Now.Sub(Start) >= MaxLatency (handler.go:180)
      flush_locked(b, false);
      continue;
    }
    b.timer_cv.wait_until(lk, steady_at(deadline));
  }
}

void make_uuid4(Batcher& b, char* dst) {
  uint64_t hi, lo;
  {
    std::lock_guard<std::mutex> lk(b.st_mu);
    hi = b.rng();
    lo = b.rng();
  }
  hi = (hi & ~0xF000ULL) | 0x4000ULL;                         // version 4
  lo = (lo & ~(0xC000ULL << 48)) | (0x8000ULL << 48);        // variant 10
  std::snprintf(dst, 40, "%08x-%04x-%04x-%04x-%012llx",
                static_cast<unsigned>(hi >> 32), static_cast<unsigned>((hi >> 16) & 0xFFFF),
                static_cast<unsigned>(hi & 0xFFFF), static_cast<unsigned>(lo >> 48),
                static_cast<unsigned long long>(lo & 0xFFFFFFFFFFFFULL));
}

void signal_fd(int fd) {
  const uint64_t one = 1;
  ssize_t r;
  do {
    r = write(fd, &one, sizeof one);
  } while (r < 0 && errno == EINTR);
}

void run_batch(Batcher& b, Batch& bt, std::vector<unsigned char>& out) {
  out.resize(static_cast<size_t>(bt.rows) * b.o_row);
  const int64_t t0 = mono_ns();
  const int rc = b.predict(b.model, bt.x.data(), b.cfg.x_dtype, bt.rows, b.cfg.n_cols,
                           b.cfg.n_cols, b.cfg.output_kind, out.data(),
                           bt.rows * b.cfg.out_width);
  const int64_t t1 = mono_ns();
  char id[40] = {0};
  if (rc == 0) {
    make_uuid4(b, id);
    for (const Waiter& w : bt.waiters)   // fan-out by index (handler.go:138-149)
      std::memcpy(w.out, out.data() + static_cast<size_t>(w.lo) * b.o_row,
                  static_cast<size_t>(w.hi - w.lo) * b.o_row);
  } else {
    const char* m = b.err ? b.err() : nullptr;   // the model thread's own last error
    std::string text = (m && *m) ? m : ("model call failed with code " + std::to_string(rc));
    std::lock_guard<std::mutex> lk(b.msg_mu);
    b.msgs[bt.seq] = std::move(text);
    b.msg_order.push_back(bt.seq);
    while (b.msg_order.size() > kMaxMessages) {
      b.msgs.erase(b.msg_order.front());
      b.msg_order.pop_front();
    }
  }
  const int64_t done = mono_ns();
  {
    std::lock_guard<std::mutex> lk(b.st_mu);
    b.st.model_ms_total += (t1 - t0) * 1e-6;
    if (rc != 0) b.st.failed_batches += 1;
  }
  bool queued = false;
  {
    std::lock_guard<std::mutex> lk(b.cq_mu);
    for (const Waiter& w : bt.waiters) {
      kb_completion c{};
      c.tag = w.tag;
      c.status = rc == 0 ? KB_OK : KB_ERR_MODEL;
      c.batch_rows = static_cast<int32_t>(bt.rows);
      c.t_done_ns = done;
      c.batch_seq = bt.seq;
      std::memcpy(c.batch_id, id, sizeof id);
      if ((c.tag & KB_TAG_CALLBACK) && b.done_fn) {
        b.done_fn(b.done_ctx, &c);   // a native caller's request (kb_set_done_callback)
      } else {
        b.cq.push_back(c);
        queued = true;
      }
    }
  }
  if (queued) signal_fd(b.efd);
}

void worker_main(Batcher* bp) {
  Batcher& b = *bp;
  std::vector<unsigned char> out;
  std::unique_lock<std::mutex> lk(b.mu);
  for (;;) {
    b.work_cv.wait(lk, [&] { return b.stop || !b.ready.empty(); });
    if (b.ready.empty()) break;   // stopping, and nothing left to run
    Batch bt = std::move(b.ready.front());
    b.ready.pop_front();
    lk.unlock();
    run_batch(b, bt, out);
    lk.lock();
    bt.x.clear();
    if (b.spare.size() < 4) b.spare.push_back(std::move(bt.x));
  }
}

// one element of a request converted into the batch's type: an IEEE cast
// (numpy's astype: round to nearest even, overflow to inf), after xgboost
// 0.82's DMatrix(list) rule when asked (scipy.sparse.csr_matrix keeps no
// zeros, so 0 is missing = NaN; a NaN it does store compares false with every
// split, i.e. always goes right = +inf; tree_model.xgb_matrix_from_list)
template <typename D, typename S>
inline D convert(S v, int transform) {
  if (transform == KB_IN_XGB_LIST) {
    if (v == S(0)) return std::numeric_limits<D>::quiet_NaN();
    if (v != v) return std::numeric_limits<D>::infinity();
  }
  return static_cast<D>(v);
}

template <typename D, typename S>
void convert_rows(unsigned char* dst, const S* src, int64_t rows, int64_t stride, int cols,
                  int transform) {
  D* d = reinterpret_cast<D*>(dst);
  for (int64_t r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) d[r * cols + c] = convert<D, S>(src[r * stride + c], transform);
}

}  // namespace

extern "C" {

int32_t kb_abi_version(void) { return KB_ABI_VERSION; }

int64_t kb_now_ns(void) { return mono_ns(); }

int kb_create(const kb_config* cfg, kb_predict_fn predict, void* model, kb_error_fn err,
              void** out) {
  if (!cfg || !predict || !out || cfg->abi_version != KB_ABI_VERSION) return KB_ERR_INVALID;
  if ((cfg->x_dtype != 0 && cfg->x_dtype != 1) || cfg->n_cols <= 0 || cfg->out_width <= 0 ||
      (cfg->out_elem_bytes != 4 && cfg->out_elem_bytes != 8) || cfg->max_inflight < 1 ||
      cfg->max_inflight > 64)
    return KB_ERR_INVALID;
  *out = nullptr;
  Batcher* b = new Batcher();
  b->cfg = *cfg;
  b->predict = predict;
  b->model = model;
  b->err = err;
  b->x_row = static_cast<size_t>(cfg->n_cols) * (cfg->x_dtype == 0 ? 4 : 8);
  b->o_row = static_cast<size_t>(cfg->out_width) * cfg->out_elem_bytes;
  b->max_rows = cfg->max_batch_rows > 0 ? cfg->max_batch_rows : 32;            // handler.go:188-190
  b->max_latency_ns = (cfg->max_latency_us > 0 ? cfg->max_latency_us : 5000 * 1000LL) * 1000LL;  // :191-193
  b->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (b->efd < 0) {
    delete b;
    return KB_ERR_SYSTEM;
  }
  try {
    b->timer = std::thread(timer_main, b);
    for (int i = 0; i < cfg->max_inflight; ++i) b->workers.emplace_back(worker_main, b);
  } catch (...) {
    {
      std::lock_guard<std::mutex> lk(b->mu);
      b->stop = true;
    }
    b->timer_cv.notify_all();
    b->work_cv.notify_all();
    if (b->timer.joinable()) b->timer.join();
    for (auto& t : b->workers) t.join();
    close(b->efd);
    delete b;
    return KB_ERR_SYSTEM;
  }
  *out = b;
  return KB_OK;
}

int kb_destroy(void* h) {
  if (!h) return KB_ERR_INVALID;
  Batcher* b = static_cast<Batcher*>(h);
  {
    std::lock_guard<std::mutex> lk(b->mu);
    flush_locked(*b, false);   // what is forming still gets answered
    b->stop = true;
  }
  b->timer_cv.notify_all();
  b->work_cv.notify_all();
  b->timer.join();
  for (auto& t : b->workers) t.join();   // workers leave once the queue is empty
  close(b->efd);
  delete b;
  return KB_OK;
}

int kb_flush(void* h) {
  if (!h) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  std::lock_guard<std::mutex> lk(b.mu);
  flush_locked(b, false);
  return KB_OK;
}

int kb_set_done_callback(void* h, kb_done_fn fn, void* ctx) {
  if (!h) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  std::lock_guard<std::mutex> lk(b.cq_mu);
  b.done_fn = fn;
  b.done_ctx = ctx;
  return KB_OK;
}

int kb_notify_fd(void* h) { return h ? static_cast<Batcher*>(h)->efd : KB_ERR_INVALID; }

int kb_submit(void* h, const void* X, int64_t rows, int64_t row_stride, void* out,
              uint64_t tag) {
  if (!h) return KB_ERR_INVALID;
  return kb_submit_convert(h, X, static_cast<Batcher*>(h)->cfg.x_dtype, rows, row_stride,
                           KB_IN_PLAIN, out, tag);
}

int kb_submit_convert(void* h, const void* X, int32_t x_dtype, int64_t rows, int64_t row_stride,
                      int32_t transform, void* out, uint64_t tag) {
  if (!h || !X || !out || rows <= 0) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  if (row_stride < b.cfg.n_cols || (x_dtype != 0 && x_dtype != 1) ||
      (transform != KB_IN_PLAIN && transform != KB_IN_XGB_LIST))
    return KB_ERR_INVALID;
  const bool copy = x_dtype == b.cfg.x_dtype && transform == KB_IN_PLAIN;
  const size_t es = b.cfg.x_dtype == 0 ? 4 : 8;
  const unsigned char* src = static_cast<const unsigned char*>(X);
  std::unique_lock<std::mutex> lk(b.mu);
  if (b.stop) return KB_ERR_CLOSED;
  Batch& f = b.forming;
  if (f.rows == 0) {
    f.start_ns = mono_ns();   // Start = the first request's arrival (handler.go:163-165)
    if (!b.spare.empty()) {
      f.x = std::move(b.spare.back());
      b.spare.pop_back();
    }
    b.timer_cv.notify_one();
  }
  const size_t at = f.x.size();
  f.x.resize(at + static_cast<size_t>(rows) * b.x_row);
  if (!copy) {
    unsigned char* dst = f.x.data() + at;
    const int nc = b.cfg.n_cols;
    if (b.cfg.x_dtype == 0 && x_dtype == 1)
      convert_rows<float, double>(dst, static_cast<const double*>(X), rows, row_stride, nc, transform);
    else if (b.cfg.x_dtype == 0)
      convert_rows<float, float>(dst, static_cast<const float*>(X), rows, row_stride, nc, transform);
    else if (x_dtype == 1)
      convert_rows<double, double>(dst, static_cast<const double*>(X), rows, row_stride, nc, transform);
    else
      convert_rows<double, float>(dst, static_cast<const float*>(X), rows, row_stride, nc, transform);
  } else if (row_stride == b.cfg.n_cols) {
    std::memcpy(f.x.data() + at, src, static_cast<size_t>(rows) * b.x_row);
  } else {
    for (int64_t r = 0; r < rows; ++r)
      std::memcpy(f.x.data() + at + static_cast<size_t>(r) * b.x_row,
                  src + static_cast<size_t>(r) * row_stride * es, b.x_row);
  }
  f.waiters.push_back({tag, static_cast<unsigned char*>(out), f.rows, f.rows + rows});
  f.rows += rows;
  if (f.rows >= b.max_rows) flush_locked(b, true);   // CurrentInputLen >= MaxBatchSize
  return KB_OK;
}

int kb_poll(void* h, kb_completion* out, int32_t cap) {
  if (!h || !out || cap <= 0) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  std::lock_guard<std::mutex> lk(b.cq_mu);
  int32_t n = 0;
  while (n < cap && !b.cq.empty()) {
    out[n++] = b.cq.front();
    b.cq.pop_front();
  }
  return n;
}

int kb_batch_message(void* h, uint64_t seq, char* buf, int32_t cap) {
  if (!h || !buf || cap <= 0) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  std::lock_guard<std::mutex> lk(b.msg_mu);
  auto it = b.msgs.find(seq);
  if (it == b.msgs.end()) return KB_ERR_INVALID;
  const size_t n = std::min(it->second.size(), static_cast<size_t>(cap - 1));
  std::memcpy(buf, it->second.data(), n);
  buf[n] = '\0';
  return static_cast<int>(n);
}

int kb_get_stats(void* h, kb_stats* st) {
  if (!h || !st) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  std::lock_guard<std::mutex> lk(b.st_mu);
  *st = b.st;
  return KB_OK;
}

int kb_loadgen(void* h, const double* arrival_s, const int32_t* rows, int64_t n,
               const void* pool, int64_t pool_rows, void* out, double* latency_ms,
               int32_t* status, int64_t* t0_ns) {
  if (!h || !arrival_s || !rows || n <= 0 || !pool || pool_rows < 128 || !out || !latency_ms ||
      !status)
    return KB_ERR_INVALID;
  for (int64_t i = 0; i < n; ++i)
    if (rows[i] < 1 || rows[i] > 64 || !(arrival_s[i] >= 0.0)) return KB_ERR_INVALID;
  Batcher& b = *static_cast<Batcher*>(h);
  const unsigned char* pl = static_cast<const unsigned char*>(pool);
  unsigned char* ob = static_cast<unsigned char*>(out);
  std::vector<int64_t> due(n);
  const int64_t t0 = mono_ns() + 20000000LL;   // 20 ms to get going
  for (int64_t i = 0; i < n; ++i) due[i] = t0 + static_cast<int64_t>(arrival_s[i] * 1e9);
  if (t0_ns) *t0_ns = t0;
  std::atomic<int64_t> left(n);
  std::thread collector([&] {
    kb_completion buf[256];
    while (left.load() > 0) {
      pollfd p{b.efd, POLLIN, 0};
      (void)poll(&p, 1, 100);
      uint64_t cnt;
      (void)!read(b.efd, &cnt, sizeof cnt);
      int k;
      while ((k = kb_poll(h, buf, 256)) > 0) {
        for (int j = 0; j < k; ++j) {
          const int64_t i = static_cast<int64_t>(buf[j].tag);
          latency_ms[i] = (buf[j].t_done_ns - due[i]) * 1e-6;
          status[i] = buf[j].status;
          left.fetch_sub(1);
        }
      }
    }
  });
  unsigned long old_slack = static_cast<unsigned long>(prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0));
  (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
  for (int64_t i = 0; i < n; ++i) {
    int64_t now = mono_ns();
    if (due[i] - now > 60000) {   // sleep to 50 us before the arrival, then spin
      const int64_t s = due[i] - 50000 - now;
      timespec ts{static_cast<time_t>(s / 1000000000LL), static_cast<long>(s % 1000000000LL)};
      nanosleep(&ts, nullptr);
    }
    while (mono_ns() < due[i]) {
    }
    const int64_t off = (i * 64) % (pool_rows - 64);
    const int rc = kb_submit(h, pl + static_cast<size_t>(off) * b.x_row, rows[i], b.cfg.n_cols,
                             ob + static_cast<size_t>(i) * 64 * b.o_row, static_cast<uint64_t>(i));
    if (rc != KB_OK) {
      status[i] = rc;
      latency_ms[i] = -1.0;
      left.fetch_sub(1);
    }
  }
  (void)prctl(PR_SET_TIMERSLACK, old_slack, 0, 0, 0);
  collector.join();
  return KB_OK;
}

}  // extern "C"
