/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see asyncpool_oracle.h for scope and parity status).
 *
 * Line-by-line restatement of src/MPIAsyncPools.jl.  Comments cite the reference line
 * each block follows.  Indices are 0-based here; the reference is 1-based.
 */
#include "asyncpool_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void set_err(orc_pool* p, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(p->errmsg, sizeof p->errmsg, fmt, ap);
  va_end(ap);
}

/* src/MPIAsyncPools.jl:35-43 (and :46 for ranks = 1:n) */
orc_pool* orc_pool_create(int64_t n, const int64_t* ranks, int64_t epoch0, int64_t nwait) {
  orc_pool* p = (orc_pool*)calloc(1, sizeof(orc_pool));
  p->n = n;
  p->ranks = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
  p->sepochs = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
  p->repochs = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
  p->active = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
  p->stimestamps = (int64_t*)calloc((size_t)(n ? n : 1), sizeof(int64_t));
  p->latency = (double*)calloc((size_t)(n ? n : 1), sizeof(double));
  p->rreq_live = (uint8_t*)calloc((size_t)(n ? n : 1), 1);
  for (int64_t i = 0; i < n; ++i) {
    p->ranks[i] = ranks ? ranks[i] : i + 1;  /* copy(ranks) / collect(1:n) */
    p->repochs[i] = epoch0;                  /* fill(epoch0, n) */
  }
  p->nwait = nwait;  /* nwait::Integer=length(ranks) -- caller passes n for the default */
  p->epoch = epoch0;
  return p;
}

void orc_pool_destroy(orc_pool* p) {
  if (!p) return;
  free(p->ranks); free(p->sepochs); free(p->repochs); free(p->active);
  free(p->stimestamps); free(p->latency); free(p->rreq_live);
  free(p);
}

/* harvest of a completed receive: :105-113 / :164-171 / :215-219 */
static void harvest(orc_pool* p, const orc_transport* tp, int64_t i, uint8_t* recvbuf,
                    const uint8_t* irecvbuf, size_t rl) {
  uint64_t now = tp->time_ns(tp->ctx);
  p->latency[i] = (double)(now - (uint64_t)p->stimestamps[i]) / 1e9;   /* :105 */
  memcpy(recvbuf + (size_t)i * rl, irecvbuf + (size_t)i * rl, rl);     /* :108 */
  p->repochs[i] = p->sepochs[i];                                        /* :109 */
}

/* dispatch: :129-138 (and the stale re-dispatch :178-183) */
static void dispatch(orc_pool* p, const orc_transport* tp, int64_t i, const uint8_t* sendbuf,
                     size_t sl, uint8_t* isendbuf, uint8_t* irecvbuf, size_t rl, int64_t tag) {
  memcpy(isendbuf + (size_t)i * sl, sendbuf, sl);         /* :130 / :178 */
  p->sepochs[i] = p->epoch;                               /* :133 / :179 */
  p->stimestamps[i] = (int64_t)tp->time_ns(tp->ctx);      /* :136 / :181 */
  tp->isend_irecv(tp->ctx, i, p->ranks[i], isendbuf + (size_t)i * sl, sl,
                  irecvbuf + (size_t)i * rl, rl, tag);    /* :137-138 / :182-183 */
  p->rreq_live[i] = 1;
}

int orc_asyncmap(orc_pool* p, const orc_transport* tp,
                 const uint8_t* sendbuf, size_t send_bytes,
                 uint8_t* recvbuf, size_t recv_bytes, size_t recv_len,
                 uint8_t* isendbuf, size_t isend_bytes,
                 uint8_t* irecvbuf, size_t irecv_bytes,
                 int nwait_kind, int64_t nwait, orc_nwait_fn fn, void* fn_ctx,
                 const char* nwait_typename, int64_t epoch, int64_t tag) {
  const int64_t comm_size = p->n;                                           /* :69 */
  if (nwait_kind == ORC_NWAIT_INT) {                                        /* :70-72 */
    if (!(0 <= nwait && nwait <= comm_size)) {
      set_err(p, "nwait must be in the range [0, length(pool.ranks)], but is %lld", (long long)nwait);
      return ORC_ARGUMENT_ERROR;
    }
  }
  /* :73-74 isbitstype checks are host-language type checks; see tests/test_oracle.py */
  if (isend_bytes != (size_t)comm_size * send_bytes) {                      /* :75 */
    set_err(p, "sendbuf is of size %zu bytes, but isendbuf is of size %zu bytes when %zu bytes are needed",
            send_bytes, isend_bytes, (size_t)comm_size * send_bytes);
    return ORC_DIMENSION_MISMATCH;
  }
  if (recv_bytes != irecv_bytes) {                                          /* :76 */
    set_err(p, "recvbuf is of size %zu bytes, but irecvbuf is of size %zu bytes", recv_bytes, irecv_bytes);
    return ORC_DIMENSION_MISMATCH;
  }
  if (comm_size == 0) { set_err(p, "DivideError: integer division error"); return ORC_ERROR; }  /* mod(x, 0) */
  if (recv_len % (size_t)comm_size != 0) {                                  /* :77 */
    set_err(p, "The length of recvbuf and irecvbuf must be a multiple of the number of workers");
    return ORC_DIMENSION_MISMATCH;
  }
  const size_t sl = send_bytes;                                             /* :80 */
  const size_t rl = irecv_bytes / (size_t)comm_size;                        /* :81 */

  p->epoch = epoch;                                                         /* :87 */
  if (tp->observe) tp->observe(tp->ctx, ORC_OBS_CALL);

  /* phase 1: harvest results received since the last call :91-114 */
  for (int64_t i = 0; i < comm_size; ++i) {
    if (!p->active[i]) continue;                                            /* :94-96 */
    if (!tp->test(tp->ctx, i)) continue;                                    /* :99-102 */
    p->rreq_live[i] = 0;
    harvest(p, tp, i, recvbuf, irecvbuf, rl);                               /* :105-109 */
    p->active[i] = 0;                                                       /* :110 */
    /* :113 MPI.Wait!(sreqs[i]) returns immediately */
  }

  /* phase 2: dispatch to every inactive worker :118-139 */
  for (int64_t i = 0; i < comm_size; ++i) {
    if (p->active[i]) continue;                                             /* :121-123 */
    p->active[i] = 1;                                                       /* :126 */
    dispatch(p, tp, i, sendbuf, sl, isendbuf, irecvbuf, rl, tag);           /* :130-138 */
  }

  /* phase 3: wait loop :145-185 */
  int64_t nrecv = 0;                                                        /* :145 */
  for (;;) {
    if (nwait_kind == ORC_NWAIT_INT) {                                      /* :148-151 */
      if (nrecv >= nwait) break;
    } else if (nwait_kind == ORC_NWAIT_FN) {                                /* :152-155 */
      int r = fn(fn_ctx, p->epoch, p->repochs, comm_size);
      if (r < 0) { set_err(p, "nwait function raised an error"); return ORC_ERROR; }
      if (r) break;
    } else {                                                                /* :156-158 */
      set_err(p, "nwait must be either an Integer or a Function, but is a %s",
              nwait_typename ? nwait_typename : "?");
      return ORC_ERROR;
    }
    int64_t i = tp->waitany(tp->ctx, comm_size, p->rreq_live);              /* :161 */
    if (i < 0) {  /* all requests null: MPI_UNDEFINED, undefined in the reference */
      set_err(p, "asyncmap!: no outstanding requests and the nwait condition is unsatisfiable");
      return ORC_ERROR;
    }
    p->rreq_live[i] = 0;
    harvest(p, tp, i, recvbuf, irecvbuf, rl);                               /* :164-168 */
    /* :171 MPI.Wait!(sreqs[i]) */
    if (p->repochs[i] == p->epoch) {                                        /* :174-176 */
      nrecv += 1;
      p->active[i] = 0;
    } else {                                                                /* :177-184 */
      dispatch(p, tp, i, sendbuf, sl, isendbuf, irecvbuf, rl, tag);
    }
  }
  return ORC_OK;                                                            /* :187 */
}

int orc_waitall(orc_pool* p, const orc_transport* tp,
                uint8_t* recvbuf, size_t recv_bytes, size_t recv_len,
                uint8_t* irecvbuf, size_t irecv_bytes) {
  const int64_t comm_size = p->n;                                           /* :196 */
  if (recv_bytes != irecv_bytes) {                                          /* :198 */
    set_err(p, "recvbuf is of size %zu bytes, but irecvbuf is of size %zu bytes", recv_bytes, irecv_bytes);
    return ORC_DIMENSION_MISMATCH;
  }
  if (comm_size == 0) { set_err(p, "DivideError: integer division error"); return ORC_ERROR; }  /* mod(x, 0) */
  if (recv_len % (size_t)comm_size != 0) {                                  /* :199 */
    set_err(p, "The length of recvbuf and irecvbuf must be a multiple of the number of workers");
    return ORC_DIMENSION_MISMATCH;
  }
  int64_t nactive = 0;                                                      /* :201 */
  for (int64_t i = 0; i < comm_size; ++i) nactive += p->active[i];
  if (nactive == 0) return ORC_OK;                                          /* :202-204 */
  const size_t rl = irecv_bytes / (size_t)comm_size;                        /* :207 */
  tp->waitall(tp->ctx, comm_size, p->rreq_live);                            /* :212 */
  for (int64_t i = 0; i < comm_size; ++i) {                                 /* :213-221 */
    if (p->active[i]) {
      p->rreq_live[i] = 0;
      harvest(p, tp, i, recvbuf, irecvbuf, rl);
      p->active[i] = 0;
    }
  }
  return ORC_OK;                                                            /* :223 */
}

/* ---------------------------------------------------------------------------------
 * Virtual-clock worker transport.  Worker protocol restated from
 * examples/iterative_example.jl:55-82 and test/kmap2.jl:76-99: each worker serves one
 * message at a time, replies exactly once per message, in FIFO order.  A task posted at
 * virtual time T completes at T + duration(worker, t) + compute_ns.
 * ------------------------------------------------------------------------------- */
struct orc_sim {
  int64_t nworkers, ncols, compute_ns;
  int kind;
  int64_t* durations;
  int64_t now;
  int64_t* t;          /* messages served by each worker (kmap2.jl:82-84) */
  int64_t* post_ns;
  int64_t* done_ns;
  int64_t* rank;
  uint8_t** rbuf;
  size_t* rl;
  uint8_t** snap;      /* bytes the worker received */
  size_t* sl;
  uint8_t* delivered;
  orc_event* ev;
  int64_t nev, capev;
  orc_obs* obs;
  int64_t nobs, capobs;
};

static void sim_log(orc_sim* s, int64_t kind, int64_t worker, int64_t t, int64_t done) {
  if (s->nobs == s->capobs) {
    s->capobs = s->capobs ? 2 * s->capobs : 1024;
    s->obs = (orc_obs*)realloc(s->obs, (size_t)s->capobs * sizeof(orc_obs));
  }
  orc_obs o = {kind, worker, t, done, s->now};
  s->obs[s->nobs++] = o;
}

orc_sim* orc_sim_create(int64_t nworkers, int kind, const int64_t* durations_ns, int64_t ncols,
                        int64_t compute_ns) {
  orc_sim* s = (orc_sim*)calloc(1, sizeof(orc_sim));
  s->nworkers = nworkers;
  s->kind = kind;
  s->ncols = ncols > 0 ? ncols : 1;
  s->compute_ns = compute_ns;
  size_t nw = (size_t)(nworkers ? nworkers : 1);
  s->durations = (int64_t*)calloc(nw * (size_t)s->ncols, sizeof(int64_t));
  if (durations_ns && ncols > 0) memcpy(s->durations, durations_ns, nw * (size_t)ncols * sizeof(int64_t));
  s->t = (int64_t*)calloc(nw, sizeof(int64_t));
  s->post_ns = (int64_t*)calloc(nw, sizeof(int64_t));
  s->done_ns = (int64_t*)calloc(nw, sizeof(int64_t));
  s->rank = (int64_t*)calloc(nw, sizeof(int64_t));
  s->rbuf = (uint8_t**)calloc(nw, sizeof(uint8_t*));
  s->rl = (size_t*)calloc(nw, sizeof(size_t));
  s->snap = (uint8_t**)calloc(nw, sizeof(uint8_t*));
  s->sl = (size_t*)calloc(nw, sizeof(size_t));
  s->delivered = (uint8_t*)calloc(nw, 1);
  s->capev = 1024;
  s->ev = (orc_event*)malloc((size_t)s->capev * sizeof(orc_event));
  return s;
}

void orc_sim_destroy(orc_sim* s) {
  if (!s) return;
  for (int64_t i = 0; i < s->nworkers; ++i) free(s->snap[i]);
  free(s->durations); free(s->t); free(s->post_ns); free(s->done_ns); free(s->rank);
  free(s->rbuf); free(s->rl); free(s->snap); free(s->sl); free(s->delivered); free(s->ev);
  free(s->obs);
  free(s);
}

static void sim_post(void* ctx, int64_t i, int64_t rank, const uint8_t* sbuf, size_t sl,
                     uint8_t* rbuf, size_t rl, int64_t tag) {
  (void)tag;
  orc_sim* s = (orc_sim*)ctx;
  s->t[i] += 1;
  s->rank[i] = rank;
  s->snap[i] = (uint8_t*)realloc(s->snap[i], sl ? sl : 1);
  memcpy(s->snap[i], sbuf, sl);   /* the worker's Irecv! receives the bytes of isendbufs[i] */
  s->sl[i] = sl;
  s->rbuf[i] = rbuf;
  s->rl[i] = rl;
  s->post_ns[i] = s->now;
  s->done_ns[i] = s->now + s->durations[i * s->ncols + (s->t[i] - 1) % s->ncols] + s->compute_ns;
  s->delivered[i] = 0;
  sim_log(s, ORC_OBS_POST, i, s->t[i], s->done_ns[i]);
}

/* the worker's reply lands in irecvbufs[i] (MPI.Isend on the worker side) */
static void sim_deliver(orc_sim* s, int64_t i) {
  if (s->delivered[i]) return;
  s->delivered[i] = 1;
  uint8_t* out = s->rbuf[i];
  size_t rl = s->rl[i];
  switch (s->kind) {
    case ORC_WORKER_ECHO: {
      size_t m = s->sl[i] < rl ? s->sl[i] : rl;
      memcpy(out, s->snap[i], m);
      memset(out + m, 0, rl - m);
      break;
    }
    case ORC_WORKER_KMAP1: {  /* test/kmap1.jl:26: sendbuf[1] = rank */
      double v = (double)s->rank[i];
      memset(out, 0, rl);
      memcpy(out, &v, rl < 8 ? rl : 8);
      break;
    }
    case ORC_WORKER_KMAP2: {  /* test/kmap2.jl:78-79,92-94: [rank, t, epoch] */
      double v[3];
      v[0] = (double)s->rank[i];
      v[1] = (double)s->t[i];
      v[2] = 0.0;
      memcpy(&v[2], s->snap[i], s->sl[i] < 8 ? s->sl[i] : 8);
      memset(out, 0, rl);
      memcpy(out, v, rl < sizeof v ? rl : sizeof v);
      break;
    }
    default: {  /* ORC_WORKER_TAG */
      int64_t v[3];
      v[0] = s->rank[i];
      v[1] = s->t[i];
      v[2] = 0;
      memcpy(&v[2], s->snap[i], s->sl[i] < 8 ? s->sl[i] : 8);
      memset(out, 0, rl);
      memcpy(out, v, rl < sizeof v ? rl : sizeof v);
      break;
    }
  }
  if (s->nev == s->capev) {
    s->capev *= 2;
    s->ev = (orc_event*)realloc(s->ev, (size_t)s->capev * sizeof(orc_event));
  }
  orc_event e = {i, s->t[i], s->post_ns[i], s->done_ns[i], s->now};
  s->ev[s->nev++] = e;
}

static int sim_test(void* ctx, int64_t i) {
  orc_sim* s = (orc_sim*)ctx;
  if (s->done_ns[i] > s->now) return 0;
  sim_deliver(s, i);
  return 1;
}

/* MPI_Waitany: the first completed live request in array order; if none has completed,
 * block until the earliest completion (ties: lowest index). */
static int64_t sim_waitany(void* ctx, int64_t n, const uint8_t* live) {
  orc_sim* s = (orc_sim*)ctx;
  int64_t best = -1;
  for (int64_t i = 0; i < n; ++i) {
    if (!live[i]) continue;
    if (s->done_ns[i] <= s->now) { sim_log(s, ORC_OBS_WAIT, -1, 0, 0); sim_deliver(s, i); return i; }
    if (best < 0 || s->done_ns[i] < s->done_ns[best]) best = i;
  }
  if (best < 0) return -1;
  s->now = s->done_ns[best];
  sim_log(s, ORC_OBS_WAIT, -1, 0, 0);
  sim_deliver(s, best);
  return best;
}

static void sim_waitall(void* ctx, int64_t n, const uint8_t* live) {
  orc_sim* s = (orc_sim*)ctx;
  int64_t tmax = s->now;
  for (int64_t i = 0; i < n; ++i)
    if (live[i] && s->done_ns[i] > tmax) tmax = s->done_ns[i];
  s->now = tmax;
  sim_log(s, ORC_OBS_WAITALL, -1, 0, 0);
  for (int64_t i = 0; i < n; ++i)
    if (live[i]) sim_deliver(s, i);
}

static void sim_observe(void* ctx, int kind) { sim_log((orc_sim*)ctx, kind, -1, 0, 0); }

static uint64_t sim_time(void* ctx) { return (uint64_t)((orc_sim*)ctx)->now; }

void orc_sim_transport(orc_sim* s, orc_transport* out) {
  out->ctx = s;
  out->isend_irecv = sim_post;
  out->test = sim_test;
  out->waitany = sim_waitany;
  out->waitall = sim_waitall;
  out->time_ns = sim_time;
  out->observe = sim_observe;
}

void orc_sim_advance(orc_sim* s, int64_t dt_ns) { s->now += dt_ns; }
int64_t orc_sim_now(const orc_sim* s) { return s->now; }
int64_t orc_sim_tasks(const orc_sim* s, int64_t worker) { return s->t[worker]; }

int64_t orc_sim_obs(const orc_sim* s, orc_obs* out, int64_t cap) {
  int64_t m = s->nobs < cap ? s->nobs : cap;
  if (out && m > 0) memcpy(out, s->obs, (size_t)m * sizeof(orc_obs));
  return s->nobs;
}

int64_t orc_sim_events(const orc_sim* s, orc_event* out, int64_t cap) {
  int64_t m = s->nev < cap ? s->nev : cap;
  if (out && m > 0) memcpy(out, s->ev, (size_t)m * sizeof(orc_event));
  return s->nev;
}
