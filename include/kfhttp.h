/*
 * kfhttp.h — the model server's HTTP/1.1 front end in native code
 * (libkfserve.so, built from kfserving_amd/csrc/kfhttp.cpp).
 *
 * Replaces, for the hot route, the tornado request path of the reference:
 *   python/kfserving/kfserving/kfserver.py:61-99   HTTPServer on the shared,
 *                                                 pre-forked socket
 *   python/kfserving/kfserving/handlers/http.py:53-95  PredictHandler.post:
 *                                                 decode -> get_model ->
 *                                                 preprocess -> validate ->
 *                                                 predict -> postprocess -> write
 * IO threads (epoll, one shared listening socket, EPOLLEXCLUSIVE accepts)
 * read and parse every request.  A request on a registered route --
 * POST /v1/models/<name>:predict whose body is {"instances": [[...]]} of the
 * model's width (kf_parse_instances) -- is answered without the interpreter:
 * its rows go to the model's native batcher (kfbatch.h, kb_submit_convert
 * with the plugin's element rule), and the batch's completion is formatted as
 * the bytes the Python server writes for it ({"message": "", "batchId": ...,
 * "predictions": [...]}, floats as Python's repr, the same status line and
 * headers).  Every other request -- other routes, other bodies, CloudEvents,
 * models without a route -- is handed to the Python application through a
 * queue signalled by an eventfd (kh_fallback_fd / kh_next_fallback), and the
 * bytes it answers are written back in order (kh_respond).  Malformed
 * requests get the Python server's 400 / 413 pages and the connection closes.
 */
#ifndef KFHTTP_H_
#define KFHTTP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KH_ABI_VERSION 1

typedef struct kh_config {
  int32_t abi_version;     /* KH_ABI_VERSION                                      */
  int32_t listen_fd;       /* a bound, listening TCP socket (KFServer.bind)       */
  int32_t io_threads;      /* >= 1                                                */
  int32_t reserved;
  int64_t max_body_bytes;  /* --max_buffer_size: larger bodies get 413            */
} kh_config;

/* A request the native side hands to the Python application.  The strings
 * stay valid until kh_respond(id) is called. */
typedef struct kh_request {
  uint64_t id;
  const char* method;      /* NUL-terminated                                      */
  const char* target;
  const char* version;
  const char* headers;     /* "name: value\n" lines, names lower-cased, in order  */
  int64_t headers_len;
  const char* body;        /* chunked bodies arrive decoded                       */
  int64_t body_len;
  int32_t keep_alive;      /* Connection != close and HTTP/1.1                    */
  int32_t reserved;
} kh_request;

typedef struct kh_stats {
  int64_t connections;     /* accepted                                            */
  int64_t native_requests; /* answered on a registered route                      */
  int64_t python_requests; /* handed to the application                           */
  int64_t bad_requests;    /* 400 / 413 answered natively                         */
} kh_stats;

int kh_create(const kh_config* cfg, void** out);

/* Answer POST /v1/models/<model>:predict natively through `batcher` (a kb_*
 * handle whose rows have n_cols columns and out_width outputs of
 * out_elem_bytes (4: float32, 8: float64) each), converting each request's
 * float64 rows with kb_submit_convert's `transform` (low 8 bits; KH_CHECK_*
 * flags above them).  The server takes the
 * batcher's done callback (kb_set_done_callback).  n_labels > 0: the
 * predictions are class indices (out_width 1), each answered with its label,
 * labels[label_offsets[i] .. label_offsets[i + 1]) being label i rendered as
 * json.dumps renders it (sklearnserver classifiers: classes_.take(index)).
 * -1 if the model already has a route. */
#define KH_CHECK_F32_FINITE (1 << 8)  /* hand to the application a body with a value
                                         that is +-inf after the float32 cast
                                         (sklearn's check_array on X.astype(float32)) */
#define KH_CHECK_NO_NAN     (1 << 9)  /* ... or holding a NaN (estimators without
                                         missing-value support)                     */
int kh_add_v1_predict(void* srv, const char* model, void* batcher, int32_t n_cols,
                      int32_t out_width, int32_t out_elem_bytes, int32_t transform,
                      const char* labels, const int32_t* label_offsets, int32_t n_labels);

/* kh_add_v1_predict for an lgbserver model: bodies are {"inputs": [{"<column>":
 * [...], ...}, ...]} (lgbserver/model.py:44-54), read into float64 rows by
 * kf_parse_inputs with the model's n_cols feature names (name j at
 * names[name_offsets[j] .. name_offsets[j + 1])); a body outside its subset
 * goes to the application.  Rows are copied as they are (KB_IN_PLAIN). */
int kh_add_v1_inputs_predict(void* srv, const char* model, void* batcher, int32_t n_cols,
                             int32_t out_width, int32_t out_elem_bytes, const char* names,
                             const int32_t* name_offsets);

/* Answer V2 tensor requests on POST /v2/models/<model>/infer natively through
 * `batcher` (the model's batcher of V2 tensor rows): a body kf_parse_v2_tensor
 * takes, of n_cols columns, is converted to the batcher's type as numpy casts
 * it (FP32 data rounded to float32 first; `transform` as kh_add_v1_predict's:
 * KB_IN_PLAIN and KH_CHECK_* flags) and answered as
 * kfserving_amd/kfserving/v2.py encode_response answers it:
 * {"model_name": ..., ["id": ...,] "outputs": [{"name": "predict", "shape":
 * [N] or [N, out_width], "datatype": "FP32" | "FP64", "data": [...]}]}.
 * Every other V2 request (binary tensor data, "outputs", other datatypes, ...)
 * goes to the application.  The route is removed with
 * kh_remove_route(srv, "v2:<model>"). */
int kh_add_v2_tensor_predict(void* srv, const char* model, void* batcher, int32_t n_cols,
                             int32_t out_width, int32_t out_elem_bytes, int32_t transform);

/* Stop answering the model natively (its requests go to the application):
 * the batcher's forming batch is flushed, the requests already submitted are
 * answered, and the batcher's done callback is detached before this returns
 * 0, so the caller may then destroy the batcher.  -2: requests were still on
 * the batcher after 20 s; the callback stays attached (late completions still
 * reach their connections), and destroying the batcher (kb_destroy answers
 * what it holds first) remains safe.  -1: no such route. */
int kh_remove_route(void* srv, const char* model);

int kh_start(void* srv);

/* Readable when kh_next_fallback has requests. */
int kh_fallback_fd(void* srv);

/* 1 and *req filled if a request was waiting, 0 if none. */
int kh_next_fallback(void* srv, kh_request* req);

/* The application's answer to request `id`: the whole serialised response
 * (status line, headers, body).  close_after: close the connection after it. */
int kh_respond(void* srv, uint64_t id, const void* data, int64_t len, int32_t close_after);

int kh_get_stats(void* srv, kh_stats* stats);

/* Stop accepting, close every connection, join the IO threads, free. */
int kh_destroy(void* srv);

/* Python's repr() of a double as json.dumps writes it (NaN, Infinity,
 * -Infinity for the specials): the length written, or -1 if cap is too small. */
int kh_repr_double(double v, char* buf, int32_t cap);

int32_t kh_abi_version(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* KFHTTP_H_ */
