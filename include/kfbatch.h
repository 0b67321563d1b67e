/*
 * kfbatch.h — the request batcher of the serving path in native code
 * (libkfserve.so, built from kfserving_amd/csrc/kfbatch.cpp).
 *
 * Replaces pkg/batcher's BatchHandler (pkg/batcher/handler.go:98-263), the Go
 * sidecar that coalesces the rows of many small `instances` requests into one
 * model call:
 *   handler.go:161-175  a request's rows are appended whole; Start is set when
 *                       the batch receives its first request
 *   handler.go:179-182  flush when CurrentInputLen >= MaxBatchSize rows, or when
 *                       Now.Sub(Start).Milliseconds() >= MaxLatency
 *   handler.go:138-149  every request gets back its own rows, by index, and the
 *                       batch's one batchId (GenerateUUID, :118)
 *   handler.go:107-116  a failed model call fans out its message to every
 *                       request of the batch, batchId ""
 *   handler.go:187-195  MaxBatchSize <= 0 -> 32, MaxLatency <= 0 -> 5000 ms
 * The model call is a function with ti_predict's signature (include/treeinfer.h),
 * so the batcher hands a batch straight to libtreeinfer without a second HTTP
 * hop, a JSON round trip or the Python interpreter.
 *
 * Deliberately different from the Go loop:
 *  - the deadline is a timed wait on CLOCK_MONOTONIC, not a 100 us poll
 *    (handler.go:33,176), and the flush test is elapsed >= MaxLatency exactly;
 *  - a flushed batch runs on one of `max_inflight` model threads while the next
 *    batch keeps forming (the Go loop runs batchPredict synchronously: no
 *    request is accepted while a batch is on the model); max_inflight = 1 and
 *    a single thread restores the serial order of batches;
 *  - requests are already float matrices (the plugin's own conversion of the
 *    request, applied per request before kb_submit), so a malformed request
 *    fails alone instead of failing the batch it would have joined.
 *
 * Completions are reported through an eventfd (kb_notify_fd) that an event
 * loop watches; kb_poll drains them.  Thread-safe: any thread may submit.
 */
#ifndef KFBATCH_H_
#define KFBATCH_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KB_ABI_VERSION 1

#define KB_OK            0
#define KB_ERR_INVALID  -1   /* bad argument (null pointer, rows <= 0, ...)      */
#define KB_ERR_CLOSED   -2   /* kb_submit after kb_destroy began                */
#define KB_ERR_SYSTEM   -3   /* eventfd / thread creation failed                */
#define KB_ERR_MODEL    -4   /* completion status: the model call failed        */

/* The model call: ti_predict (include/treeinfer.h) or a function of the same
 * signature.  Returns 0 on success. */
typedef int (*kb_predict_fn)(void* model, const void* X, int32_t x_dtype, int64_t n_rows,
                             int32_t n_cols, int64_t row_stride, int32_t output_kind,
                             void* out, int64_t out_len);
/* Text of the last failure on the calling thread (ti_last_error); may be NULL. */
typedef const char* (*kb_error_fn)(void);

typedef struct kb_config {
  int32_t abi_version;     /* KB_ABI_VERSION                                     */
  int32_t x_dtype;         /* TI_F32 (0) or TI_F64 (1): the element type of X    */
  int32_t n_cols;          /* features per row                                   */
  int32_t output_kind;     /* passed through to the model call                   */
  int32_t out_width;       /* output elements per row                            */
  int32_t out_elem_bytes;  /* 4 or 8                                             */
  int64_t max_batch_rows;  /* MaxBatchSize (<= 0: 32, handler.go:34)             */
  int64_t max_latency_us;  /* MaxLatency in microseconds (<= 0: 5000 ms, :35)    */
  int32_t max_inflight;    /* model threads: batches on the model at once (>= 1) */
  int32_t reserved;
} kb_config;

typedef struct kb_completion {
  uint64_t tag;            /* the tag passed to kb_submit                        */
  int32_t status;          /* KB_OK, or KB_ERR_MODEL (kb_batch_message)          */
  int32_t batch_rows;      /* rows of the batch that answered this request       */
  int64_t t_done_ns;       /* CLOCK_MONOTONIC when its rows were written         */
  uint64_t batch_seq;      /* 1, 2, ... in flush order                           */
  char batch_id[40];       /* UUID v4 of the batch; "" when the model failed     */
} kb_completion;

typedef struct kb_stats {
  int64_t batches;         /* batches flushed                                    */
  int64_t rows;            /* rows flushed                                       */
  int64_t max_batch_rows;  /* largest batch                                      */
  int64_t full_flushes;    /* flushed by MaxBatchSize                            */
  int64_t timer_flushes;   /* flushed by MaxLatency                              */
  int64_t failed_batches;  /* model calls that failed                            */
  double  model_ms_total;  /* wall time inside the model call, summed            */
} kb_stats;

/* Start a batcher in front of `predict(model, ...)`.  `err` may be NULL. */
int kb_create(const kb_config* cfg, kb_predict_fn predict, void* model, kb_error_fn err,
              void** out);

/* Flush what is forming, wait for every batch on the model, post their
 * completions, stop the threads and free the handle.  Completions not yet
 * polled are discarded with it. */
int kb_destroy(void* batcher);

/* Flush the forming batch now, whatever its size and age (a server draining
 * its requests before it stops). */
int kb_flush(void* batcher);

/* The eventfd that becomes readable when completions are waiting (read its
 * 8-byte counter to re-arm it, then kb_poll until it returns 0). */
int kb_notify_fd(void* batcher);

/* Queue one request: `rows` rows of X (row_stride elements apart) are copied
 * into the forming batch before the call returns, so X may be freed at once.
 * `out` (rows * out_width elements of out_elem_bytes) must stay valid until
 * the request's completion is polled; the request's rows of the batch's
 * output are written there.  The request may flush the batch (MaxBatchSize). */
int kb_submit(void* batcher, const void* X, int64_t rows, int64_t row_stride, void* out,
              uint64_t tag);

/* kb_submit for a request whose rows are of another element type or still
 * need the plugin's conversion: each element is converted while it is copied
 * into the batch (an IEEE cast, numpy's astype), after `transform`:
 *   KB_IN_PLAIN      the value as it is;
 *   KB_IN_XGB_LIST   xgboost 0.82's DMatrix(list) (xgbserver/model.py:46): the
 *                    scipy.sparse conversion keeps no zeros, so 0 is missing
 *                    (NaN), and a stored NaN never satisfies x < split (+inf).
 * x_dtype: TI_F32 (0) or TI_F64 (1). */
#define KB_IN_PLAIN     0
#define KB_IN_XGB_LIST  1
int kb_submit_convert(void* batcher, const void* X, int32_t x_dtype, int64_t rows,
                      int64_t row_stride, int32_t transform, void* out, uint64_t tag);

/* Completions of requests whose tag has KB_TAG_CALLBACK set go to `fn`,
 * called on a model thread (with the batcher's completion lock held: it must
 * not call back into the batcher), instead of the kb_poll queue; the native
 * HTTP front end (include/kfhttp.h) answers its connections this way while
 * the event loop polls the same batcher for its own requests.  NULL fn: every
 * completion is queued. */
#define KB_TAG_CALLBACK (1ULL << 63)
typedef void (*kb_done_fn)(void* ctx, const kb_completion* c);
int kb_set_done_callback(void* batcher, kb_done_fn fn, void* ctx);

/* Move up to `cap` completions into `out`; returns how many (0: none). */
int kb_poll(void* batcher, kb_completion* out, int32_t cap);

/* The model's error text for a failed batch (status KB_ERR_MODEL), copied
 * into buf (NUL-terminated); the length, or KB_ERR_INVALID if unknown. */
int kb_batch_message(void* batcher, uint64_t batch_seq, char* buf, int32_t cap);

int kb_get_stats(void* batcher, kb_stats* stats);

/* CLOCK_MONOTONIC in nanoseconds (the clock of t_done_ns; Python's
 * time.monotonic() reads the same clock). */
int64_t kb_now_ns(void);

/* Open-loop load for measurement (bench.py's batched-latency leg): request i
 * of `rows[i]` rows, taken from `pool` (pool_rows dense rows) at row
 * (i * 64) mod (pool_rows - 64), is submitted at t0 + arrival_s[i] (a
 * timed sleep, then a spin for the last 50 us), from this thread, while a
 * second thread collects completions.  Its output goes to `out` at element
 * offset i * 64 * out_width.  latency_ms[i] = completion - scheduled arrival.
 * Returns KB_OK once every request completed; *t0_ns receives t0.  The
 * caller must not poll this batcher meanwhile. */
int kb_loadgen(void* batcher, const double* arrival_s, const int32_t* rows, int64_t n,
               const void* pool, int64_t pool_rows, void* out, double* latency_ms,
               int32_t* status, int64_t* t0_ns);

int32_t kb_abi_version(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* KFBATCH_H_ */
