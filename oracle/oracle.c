/*
 * oracle.c — CPU restatement of the ruserf hot path.  TEST INFRASTRUCTURE:
 * see the header of oracle.h.  Every function cites the reference file:line
 * it restates (paths relative to the al8n/ruserf repository root).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, so that a*b+c is never
 * contracted into an FMA: Rust does not contract either).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 constants)               */
/* ------------------------------------------------------------------------ */
void orc_philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* purpose tags in ctr[1] bits 24..31 */
#define PURPOSE_UNIT 1u
#define PURPOSE_PEER 2u
#define PURPOSE_VPROBE 3u
#define PURPOSE_NBR 5u
#define PURPOSE_POS 6u

static inline void seed_key(uint64_t seed, uint32_t key[2]) {
  key[0] = (uint32_t)seed;
  key[1] = (uint32_t)(seed >> 32);
}
static inline uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

/* ------------------------------------------------------------------------ */
/* Rust std semantics                                                       */
/* ------------------------------------------------------------------------ */
/* Duration::as_secs_f64 = secs as f64 + nanos as f64 / 1e9 */
double orc_as_secs_f64(uint64_t ns) {
  uint64_t secs = ns / 1000000000ull;
  uint32_t nanos = (uint32_t)(ns % 1000000000ull);
  return (double)secs + (double)nanos / 1e9;
}
/* `f64 as u64`: truncate toward zero, saturate, NaN -> 0 */
static inline uint64_t sat_u64(double x) {
  if (!(x > 0.0)) return 0;
  if (x >= 18446744073709551616.0) return UINT64_MAX;
  return (uint64_t)x;
}
/* f64::max / f64::min: return the non-NaN operand (== C99 fmax/fmin) */
static inline double rmax(double a, double b) { return fmax(a, b); }
static inline double rmin(double a, double b) { return fmin(a, b); }

/* ------------------------------------------------------------------------ */
/* Vivaldi: Coordinate / helpers  (core/src/coordinate.rs)                  */
/* ------------------------------------------------------------------------ */
/* CoordinateOptions::new  coordinate.rs:200-213 */
void orc_coord_opts_default(orc_coord_opts* o) {
  memset(o, 0, sizeof(*o));
  o->dimensionality = 8;
  o->vivaldi_error_max = 1.5;
  o->vivaldi_ce = 0.25;
  o->vivaldi_cc = 0.25;
  o->adjustment_window_size = 20;
  o->height_min = 10.0e-6;
  o->latency_filter_size = 3;
  o->gravity_rho = 150.0;
}

/* Coordinate::with_options  coordinate.rs:568-577 */
void orc_coord_with_options(const orc_coord_opts* o, orc_coord* c) {
  memset(c, 0, sizeof(*c));
  c->dim = o->dimensionality;
  c->error = o->vivaldi_error_max;
  c->adjustment = 0.0;
  c->height = o->height_min;
}

/* Coordinate::is_valid  coordinate.rs:581-586 */
int orc_coord_is_valid(const orc_coord* c) {
  for (uint32_t i = 0; i < c->dim; ++i)
    if (!isfinite(c->portion[i])) return 0;
  return isfinite(c->error) && isfinite(c->adjustment) && isfinite(c->height);
}

/* magnitude_in_place  coordinate.rs:779-781: fold(0.0, acc + x*x).sqrt() */
double orc_magnitude(const double* v, uint32_t n) {
  double acc = 0.0;
  for (uint32_t i = 0; i < n; ++i) acc = acc + v[i] * v[i];
  return sqrt(acc);
}

/* raw_distance_to  coordinate.rs:647-649 */
double orc_coord_raw_distance(const orc_coord* a, const orc_coord* b) {
  double acc = 0.0;
  for (uint32_t i = 0; i < a->dim; ++i) {
    double d = a->portion[i] - b->portion[i];
    acc = acc + d * d;
  }
  return sqrt(acc) + a->height + b->height;
}

/* distance_to  coordinate.rs:630-644 -> Duration nanoseconds */
uint64_t orc_coord_distance_ns(const orc_coord* a, const orc_coord* b) {
  double dist = orc_coord_raw_distance(a, b);
  double adjusted = dist + a->adjustment + b->adjustment;
  double d = adjusted > 0.0 ? adjusted : dist;
  return sat_u64(d * 1.0e9);
}

/* rand_f64  coordinate.rs:812-821 (thread_rng replaced by Philox) */
double orc_rand_f64(orc_rng* r) {
  for (;;) {
    uint32_t ctr[4] = {r->draw++, (PURPOSE_UNIT << 24) | (r->call & 0xFFFFFFu), r->member, r->round};
    uint32_t o[4];
    orc_philox4x32(ctr, r->key, o);
    uint64_t u = (((uint64_t)o[1] << 32) | o[0]) & 0x7FFFFFFFFFFFFFFFull;
    double f = (double)u / 9223372036854775808.0;
    if (f == 1.0) continue;
    return f;
  }
}

/* unit_vector_at  coordinate.rs:786-810 */
double orc_unit_vector_at(const double* v1, const double* v2, uint32_t n, double* ret, orc_rng* r) {
  for (uint32_t i = 0; i < n; ++i) ret[i] = v1[i] - v2[i];
  double mag = orc_magnitude(ret, n);
  if (mag > 1.0e-6) {
    double rc = 1.0 / mag;
    for (uint32_t i = 0; i < n; ++i) ret[i] *= rc;
    return mag;
  }
  for (uint32_t i = 0; i < n; ++i) ret[i] = orc_rand_f64(r) - 0.5;
  mag = orc_magnitude(ret, n);
  if (mag > 1.0e-6) {
    double rc = 1.0 / mag;
    for (uint32_t i = 0; i < n; ++i) ret[i] *= rc;
    return 0.0;
  }
  for (uint32_t i = 0; i < n; ++i) ret[i] = 0.0;
  ret[0] = 1.0;
  return 0.0;
}

/* apply_force_in_place  coordinate.rs:614-626 */
void orc_apply_force_in_place(orc_coord* self, double height_min, double force,
                              const orc_coord* other, orc_rng* r) {
  double unit[ORC_MAX_DIM];
  double mag = orc_unit_vector_at(self->portion, other->portion, self->dim, unit, r);
  for (uint32_t i = 0; i < self->dim; ++i) unit[i] *= force;        /* mul_in_place */
  for (uint32_t i = 0; i < self->dim; ++i) self->portion[i] += unit[i]; /* add_in_place */
  if (mag > 1.0e-6) {
    self->height = (self->height + other->height) * force / mag + self->height;
    self->height = rmax(self->height, height_min);
  }
}

/* ------------------------------------------------------------------------ */
/* CoordinateClient  coordinate.rs:252-500                                  */
/* ------------------------------------------------------------------------ */
/* latency_filter  coordinate.rs:292-307: push, trim front, median of sorted copy */
static double latency_filter_core(orc_filter* f, uint32_t fsize, double rtt_seconds) {
  f->s[f->len++] = rtt_seconds;
  if (f->len > fsize) {
    memmove(&f->s[0], &f->s[1], sizeof(double) * (f->len - 1));
    f->len--;
  }
  double tmp[ORC_MAX_FILTER + 1];
  uint32_t n = f->len;
  memcpy(tmp, f->s, sizeof(double) * n);
  for (uint32_t i = 1; i < n; ++i) { /* any correct sort: equal keys are equal values */
    double v = tmp[i];
    uint32_t j = i;
    while (j > 0 && tmp[j - 1] > v) {
      tmp[j] = tmp[j - 1];
      --j;
    }
    tmp[j] = v;
  }
  return tmp[n / 2];
}

typedef struct {
  orc_coord* coord;
  const orc_coord* origin;
  const orc_coord_opts* opts;
  double* adj_samples;
  uint32_t* adj_index;
  uint64_t* resets;
} client_view;

/* update_vivaldi  coordinate.rs:311-330 */
static void update_vivaldi(client_view* c, const orc_coord* other, double rtt_seconds, orc_rng* r) {
  orc_coord* me = c->coord;
  double dist = orc_as_secs_f64(orc_coord_distance_ns(me, other));
  rtt_seconds = rmax(rtt_seconds, 1.0e-6);
  double wrongness = fabs((dist - rtt_seconds) / rtt_seconds);
  double total_error = rmax(me->error + other->error, 1.0e-6);
  double weight = me->error / total_error;
  me->error = rmin((c->opts->vivaldi_ce * weight * wrongness) +
                       (me->error * (1.0 - c->opts->vivaldi_ce * weight)),
                   c->opts->vivaldi_error_max);
  double force = c->opts->vivaldi_cc * weight * (rtt_seconds - dist);
  r->call = 0;
  r->draw = 0;
  orc_apply_force_in_place(me, c->opts->height_min, force, other, r);
}

/* update_adjustment  coordinate.rs:334-346 */
static void update_adjustment(client_view* c, const orc_coord* other, double rtt_seconds) {
  uint32_t w = c->opts->adjustment_window_size;
  if (w == 0) return;
  double dist = orc_coord_raw_distance(c->coord, other);
  c->adj_samples[*c->adj_index] = rtt_seconds - dist;
  *c->adj_index = (*c->adj_index + 1) % w;
  double sum = 0.0;
  for (uint32_t i = 0; i < w; ++i) sum = sum + c->adj_samples[i];
  c->coord->adjustment = sum / (2.0 * (double)w);
}

/* update_gravity  coordinate.rs:283-289 */
static void update_gravity(client_view* c, orc_rng* r) {
  uint64_t secs = orc_coord_distance_ns(c->origin, c->coord) / 1000000000ull; /* as_secs */
  double x = (double)secs / c->opts->gravity_rho;
  double force = -1.0 * (x * x); /* f64::powf(x, 2.0) == x*x (correctly rounded) */
  r->call = 1;
  r->draw = 0;
  orc_apply_force_in_place(c->coord, c->opts->height_min, force, c->origin, r);
}

/* check_coordinate  coordinate.rs:436-446 */
static int check_coordinate(const orc_coord* me, const orc_coord* other) {
  if (me->dim != other->dim) return ORC_ERR_DIM_MISMATCH;
  if (!orc_coord_is_valid(other)) return ORC_ERR_INVALID_COORD;
  return ORC_OK;
}

/* CoordinateClient::update  coordinate.rs:462-499 */
static int client_update_core(client_view* c, orc_filter* filt, const orc_coord* other,
                              uint64_t rtt_ns, orc_rng* r) {
  int e = check_coordinate(c->coord, other);
  if (e) return e;
  if (rtt_ns > 10000000000ull) return ORC_ERR_INVALID_RTT; /* rtt > MAX_RTT (10 s) */
  double rtt_seconds = latency_filter_core(filt, c->opts->latency_filter_size, orc_as_secs_f64(rtt_ns));
  update_vivaldi(c, other, rtt_seconds, r);
  update_adjustment(c, other, rtt_seconds);
  update_gravity(c, r);
  if (!orc_coord_is_valid(c->coord)) {
    (*c->resets)++;
    orc_coord_with_options(c->opts, c->coord);
  }
  return ORC_OK;
}

/* CoordinateClient::with_options  coordinate.rs:388-402 */
int orc_client_init(orc_client* c, const orc_coord_opts* o, uint32_t n_slots) {
  if (o->dimensionality == 0 || o->dimensionality > ORC_MAX_DIM) return -1;
  if (o->adjustment_window_size > ORC_MAX_WINDOW) return -1;
  if (o->latency_filter_size == 0 || o->latency_filter_size > ORC_MAX_FILTER) return -1;
  memset(c, 0, sizeof(*c));
  c->opts = *o;
  orc_coord_with_options(o, &c->coord);
  orc_coord_with_options(o, &c->origin);
  c->n_slots = n_slots;
  c->filters = (orc_filter*)calloc(n_slots ? n_slots : 1, sizeof(orc_filter));
  return c->filters ? 0 : -1;
}
void orc_client_free(orc_client* c) {
  free(c->filters);
  c->filters = NULL;
}
/* set_coordinate  coordinate.rs:412-415 */
int orc_client_set_coordinate(orc_client* c, const orc_coord* coord) {
  int e = check_coordinate(&c->coord, coord);
  if (e) return e;
  c->coord = *coord;
  return ORC_OK;
}
/* forget_node  coordinate.rs:455-457 */
void orc_client_forget_node(orc_client* c, uint32_t slot) {
  if (slot < c->n_slots) c->filters[slot].len = 0;
}
double orc_client_latency_filter(orc_client* c, uint32_t slot, double rtt_seconds) {
  return latency_filter_core(&c->filters[slot], c->opts.latency_filter_size, rtt_seconds);
}
int orc_client_update(orc_client* c, uint32_t slot, const orc_coord* other, uint64_t rtt_ns,
                      orc_rng* rng, orc_coord* out) {
  if (slot >= c->n_slots) return -1;
  client_view v = {&c->coord, &c->origin, &c->opts, c->adjustment_samples, &c->adjustment_index, &c->resets};
  int e = client_update_core(&v, &c->filters[slot], other, rtt_ns, rng);
  if (!e && out) *out = c->coord;
  return e;
}

/* ------------------------------------------------------------------------ */
/* Vivaldi population rounds (synthetic network of BASELINE configs 1 & 5)  */
/* ------------------------------------------------------------------------ */
uint32_t orc_row_stride(uint32_t dim) { return ((dim + 3 + 3) / 4) * 4; }

static inline void row_to_coord(const double* row, uint32_t dim, orc_coord* c) {
  memset(c, 0, sizeof(*c));
  c->dim = dim;
  for (uint32_t i = 0; i < dim; ++i) c->portion[i] = row[i];
  c->error = row[dim];
  c->adjustment = row[dim + 1];
  c->height = row[dim + 2];
}
static inline void coord_to_row(const orc_coord* c, double* row) {
  for (uint32_t i = 0; i < c->dim; ++i) row[i] = c->portion[i];
  row[c->dim] = c->error;
  row[c->dim + 1] = c->adjustment;
  row[c->dim + 2] = c->height;
}

void orc_gen_neighbors(uint64_t seed, uint32_t n, uint32_t peers, uint32_t* nbr) {
  uint32_t key[2];
  seed_key(seed, key);
  for (uint32_t m = 0; m < n; ++m)
    for (uint32_t q = 0; q < peers; ++q) {
      uint32_t ctr[4] = {q, PURPOSE_NBR << 24, m, 0}, o[4];
      orc_philox4x32(ctr, key, o);
      uint32_t p = mulhi32(o[0], n - 1);
      if (p >= m) p++;
      nbr[(size_t)m * peers + q] = p;
    }
}

/* ground-truth position of member m: x,y ~ U[0,0.05) s, h ~ U[0,0.002) s */
void orc_true_position(uint64_t seed, uint32_t m, double* x, double* y, double* h) {
  uint32_t key[2];
  seed_key(seed, key);
  uint32_t ctr[4] = {0, PURPOSE_POS << 24, m, 0}, o[4];
  orc_philox4x32(ctr, key, o);
  const double s32 = 2.3283064365386963e-10; /* 2^-32 */
  *x = ((double)o[0] * s32) * 0.05;
  *y = ((double)o[1] * s32) * 0.05;
  *h = ((double)o[2] * s32) * 0.002;
}

void orc_vivaldi_probe(uint64_t seed, uint32_t n, uint32_t peers, const uint32_t* nbr, uint32_t m,
                       uint32_t round, uint32_t* slot_out, uint64_t* rtt_out) {
  (void)n;
  uint32_t key[2];
  seed_key(seed, key);
  uint32_t ctr[4] = {0, PURPOSE_VPROBE << 24, m, round}, o[4];
  orc_philox4x32(ctr, key, o);
  /* memberlist's probe loop walks its member list round-robin (state.go probe():
     probeIndex advances one node per probe interval; memberlist is a dependency
     not vendored in /root/reference): slot = round mod peers over the member's
     fixed, Philox-drawn neighbour list.  o[1] is the RTT jitter. */
  uint32_t q = round % peers;
  uint32_t p = nbr[(size_t)m * peers + q];
  double xm, ym, hm, xp, yp, hp;
  orc_true_position(seed, m, &xm, &ym, &hm);
  orc_true_position(seed, p, &xp, &yp, &hp);
  double dx = xm - xp, dy = ym - yp;
  double d = sqrt(dx * dx + dy * dy) + hm + hp;
  double jit = 1.0 + 0.1 * ((double)o[1] * 2.3283064365386963e-10);
  *slot_out = q;
  *rtt_out = sat_u64((d * jit) * 1.0e9);
}

int orc_vivaldi_pop_init(orc_vivaldi_pop* p, uint32_t n, uint32_t peers, const orc_coord_opts* o,
                         uint64_t seed) {
  memset(p, 0, sizeof(*p));
  if (n < 2 || peers == 0 || o->dimensionality == 0 || o->dimensionality > ORC_MAX_DIM) return -1;
  if (o->adjustment_window_size > ORC_MAX_WINDOW) return -1;
  if (o->latency_filter_size == 0 || o->latency_filter_size > ORC_MAX_FILTER) return -1;
  p->n = n;
  p->peers = peers;
  p->opts = *o;
  p->seed = seed;
  p->row_stride = orc_row_stride(o->dimensionality);
  size_t rows = (size_t)n * p->row_stride;
  p->rows_cur = (double*)calloc(rows, sizeof(double));
  p->rows_nxt = (double*)calloc(rows, sizeof(double));
  p->adj = (double*)calloc((size_t)n * (o->adjustment_window_size ? o->adjustment_window_size : 1), sizeof(double));
  p->adj_idx = (uint32_t*)calloc(n, sizeof(uint32_t));
  p->filt = (double*)calloc((size_t)n * peers * o->latency_filter_size, sizeof(double));
  p->filt_len = (uint32_t*)calloc((size_t)n * peers, sizeof(uint32_t));
  p->nbr = (uint32_t*)calloc((size_t)n * peers, sizeof(uint32_t));
  if (!p->rows_cur || !p->rows_nxt || !p->adj || !p->adj_idx || !p->filt || !p->filt_len || !p->nbr) {
    orc_vivaldi_pop_free(p);
    return -1;
  }
  orc_coord c;
  orc_coord_with_options(o, &c);
  for (uint32_t m = 0; m < n; ++m) coord_to_row(&c, p->rows_cur + (size_t)m * p->row_stride);
  orc_gen_neighbors(seed, n, peers, p->nbr);
  return 0;
}

void orc_vivaldi_pop_free(orc_vivaldi_pop* p) {
  free(p->rows_cur);
  free(p->rows_nxt);
  free(p->adj);
  free(p->adj_idx);
  free(p->filt);
  free(p->filt_len);
  free(p->nbr);
  memset(p, 0, sizeof(*p));
}

typedef struct {
  orc_vivaldi_pop* p;
  uint32_t round, lo, hi;
  uint64_t resets;
  const double* stale;   /* NULL, or the rows of the last table refresh (members outside shard_n) */
  uint32_t shard_n;
} viv_job;

/* the row member m reads for peer `peer`: the previous round's, or (stale != NULL, peer in
 * another shard of shard_n members) the row as of the last refresh of the table */
static inline const double* viv_peer_row(const orc_vivaldi_pop* p, const double* stale, uint32_t shard_n, uint32_t m,
                                         uint32_t peer) {
  if (stale && peer / shard_n != m / shard_n) return stale + (size_t)peer * p->row_stride;
  return p->rows_cur + (size_t)peer * p->row_stride;
}

static void viv_member(orc_vivaldi_pop* p, uint32_t m, uint32_t round, uint64_t* resets, const double* stale,
                       uint32_t shard_n) {
  const uint32_t dim = p->opts.dimensionality, F = p->opts.latency_filter_size;
  const uint32_t W = p->opts.adjustment_window_size;
  uint32_t slot;
  uint64_t rtt;
  orc_vivaldi_probe(p->seed, p->n, p->peers, p->nbr, m, round, &slot, &rtt);
  uint32_t peer = p->nbr[(size_t)m * p->peers + slot];
  orc_coord me, other, origin;
  row_to_coord(p->rows_cur + (size_t)m * p->row_stride, dim, &me);
  row_to_coord(viv_peer_row(p, stale, shard_n, m, peer), dim, &other);
  orc_coord_with_options(&p->opts, &origin);
  /* filter (Vec semantics) over the flat [n][peers][F] store */
  orc_filter f;
  size_t fi = (size_t)m * p->peers + slot;
  f.len = p->filt_len[fi];
  memcpy(f.s, p->filt + fi * F, sizeof(double) * F);
  double* adj = W ? p->adj + (size_t)m * W : NULL;
  client_view v = {&me, &origin, &p->opts, adj, &p->adj_idx[m], resets};
  orc_rng r;
  seed_key(p->seed, r.key);
  r.member = m;
  r.round = round;
  r.call = 0;
  r.draw = 0;
  client_update_core(&v, &f, &other, rtt, &r);
  memcpy(p->filt + fi * F, f.s, sizeof(double) * F);
  p->filt_len[fi] = f.len;
  double* out = p->rows_nxt + (size_t)m * p->row_stride;
  memset(out, 0, sizeof(double) * p->row_stride);
  coord_to_row(&me, out);
}

static void* viv_worker(void* arg) {
  viv_job* j = (viv_job*)arg;
  for (uint32_t m = j->lo; m < j->hi; ++m) viv_member(j->p, m, j->round, &j->resets, j->stale, j->shard_n);
  return NULL;
}

static int viv_rounds(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads, double* stale,
                      uint32_t shard_n, uint32_t refresh_every);
int orc_vivaldi_pop_rounds(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads) {
  return viv_rounds(p, round0, rounds, nthreads, NULL, p->n, 1);
}
int orc_vivaldi_pop_rounds_stale(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads, double* stale,
                                 uint32_t shard_n, uint32_t refresh_every) {
  if (!stale || shard_n == 0 || refresh_every == 0) return -1;
  return viv_rounds(p, round0, rounds, nthreads, stale, shard_n, refresh_every);
}
static int viv_rounds(orc_vivaldi_pop* p, uint32_t round0, uint32_t rounds, int nthreads, double* stale,
                      uint32_t shard_n, uint32_t refresh_every) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  viv_job jobs[256];
  for (uint32_t t = round0; t < round0 + rounds; ++t) {
    uint32_t per = (p->n + nthreads - 1) / nthreads;
    int launched = 0;
    for (int i = 0; i < nthreads; ++i) {
      uint32_t lo = (uint32_t)i * per, hi = lo + per;
      if (hi > p->n) hi = p->n;
      jobs[i].p = p;
      jobs[i].round = t;
      jobs[i].lo = lo < p->n ? lo : p->n;
      jobs[i].hi = hi;
      jobs[i].resets = 0;
      jobs[i].stale = stale;
      jobs[i].shard_n = shard_n;
      if (nthreads == 1) {
        viv_worker(&jobs[i]);
      } else {
        pthread_create(&th[i], NULL, viv_worker, &jobs[i]);
        launched++;
      }
    }
    for (int i = 0; i < launched; ++i) pthread_join(th[i], NULL);
    for (int i = 0; i < nthreads; ++i) p->resets += jobs[i].resets;
    double* tmp = p->rows_cur;
    p->rows_cur = p->rows_nxt;
    p->rows_nxt = tmp;
    /* the table refresh (an all-gather of every shard's rows) after every refresh_every-th round */
    if (stale && (t + 1) % refresh_every == 0) memcpy(stale, p->rows_cur, sizeof(double) * (size_t)p->n * p->row_stride);
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Gossip world: member-state merge + dissemination                         */
/* ------------------------------------------------------------------------ */
#define EMPTY_RUMOR 0xFFFFFFFFu

/* memberlist retransmitLimit: mult * ceil(log10(n+1))  (un-vendored; restated) */
uint32_t orc_retransmit_limit(uint32_t mult, uint64_t n) {
  uint64_t x = n + 1, p = 1;
  uint32_t d = 0;
  while (p < x) {
    p *= 10;
    d++;
  }
  return mult * d;
}

static uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) {
    v >>= 7;
    n++;
  }
  return n;
}

/* Encoded message length model (types/src/{join,leave,user_event,query}.rs
 * encoded_len: u32 length prefix + varint ltime + fields; +1 type byte).  A
 * node id is modelled as a 12-byte encoded SmolStr. */
uint32_t orc_msg_len(uint8_t type, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  uint32_t base = 1 + 4 + varint_len(ltime);
  switch (type) {
    case ORC_MSG_JOIN: return base + 12;
    case ORC_MSG_LEAVE: return base + 12 + 1;
    case ORC_MSG_USER_EVENT: return base + (4 + name_len) + (4 + payload_len) + 1;
    case ORC_MSG_QUERY: return base + 4 + 28 + 4 + 1 + 8 + (4 + name_len) + (4 + payload_len);
    default: return base;
  }
}

/* Serf::user_event  api.rs:255-287: name + payload against max_user_event_size
 * (UserEventLimitTooLarge), then USER_EVENT_SIZE_LIMIT (UserEventTooLarge); then the
 * encoded length (message_encoded_len: the model's length without the type byte) against
 * both (RawUserEventTooLarge) -- all before event_clock.increment (api.rs:301) */
int32_t orc_user_event_check(uint32_t max_ue, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  uint64_t before = (uint64_t)name_len + payload_len;
  if (before > max_ue) return ORC_E_UE_LIMIT;
  if (before > ORC_USER_EVENT_SIZE_LIMIT) return ORC_E_UE_TOO_LARGE;
  uint32_t len = orc_msg_len(ORC_MSG_USER_EVENT, ltime, name_len, payload_len) - 1;
  if (len > max_ue) return ORC_E_UE_RAW;
  if (len > ORC_USER_EVENT_SIZE_LIMIT) return ORC_E_UE_RAW;
  return 0;
}

/* query_in  base.rs:916-921: the encoded query against query_size_limit (QueryTooLarge),
 * before anything is registered or queued */
int32_t orc_query_check(uint32_t limit, uint64_t ltime, uint32_t name_len, uint32_t payload_len) {
  if ((uint64_t)name_len + payload_len > limit) return ORC_E_QUERY_TOO_LARGE; /* encoding holds both */
  uint32_t len = orc_msg_len(ORC_MSG_QUERY, ltime, name_len, payload_len) - 1;
  if (len > limit) return ORC_E_QUERY_TOO_LARGE;
  return 0;
}

int orc_world_action_status(const orc_world* w, int32_t* out, uint32_t n) {
  if (n > w->last_n_acts) return -1;
  if (n) memcpy(out, w->act_status, (size_t)n * sizeof(int32_t));
  return 0;
}

uint64_t orc_digest_mix(uint64_t d, uint64_t x) {
  d ^= x;
  d *= 0x100000001B3ull;
  d ^= d >> 29;
  return d;
}

#define DIG_USER 0x1000000000000000ull
#define DIG_QUERY 0x2000000000000000ull
#define DIG_MEMBER 0x3000000000000000ull
enum { EV_JOIN = 0, EV_LEAVE = 1, EV_FAILED = 2, EV_REAP = 3, EV_UPDATE = 4 };

/* the snapshotter's process_member_event (snapshot.rs:686-711): Join adds the node to
 * the alive set, Leave / Failed remove it; nothing is recorded after a leave */
static inline void snap_member_event(orc_world* w, uint32_t m, uint32_t ev, uint32_t subj) {
  if (!w->snap_bits || (w->snap_sn[(size_t)m * 4 + 3] & 1)) return;
  uint32_t* word = w->snap_bits + (size_t)m * w->snap_w + (subj >> 5);
  if (ev == EV_JOIN) *word |= 1u << (subj & 31);
  else if (ev == EV_LEAVE || ev == EV_FAILED) *word &= ~(1u << (subj & 31));
}

static void dlog_put(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key, uint64_t flags);
/* a MemberEvent sent to the application (event_tx): the order-sensitive digest, the
 * snapshotter, and the delivery log (flags word ORC_LOG_MEMBER, time word = the type, key =
 * subject), so the log is the member's whole event stream in production order */
static inline void digest_member_event(orc_world* w, uint32_t m, uint32_t ev, uint32_t subj) {
  w->digest[m] = orc_digest_mix(w->digest[m], DIG_MEMBER | ((uint64_t)ev << 32) | subj);
  snap_member_event(w, m, ev, subj);
  dlog_put(w, m, ev, subj, ORC_LOG_MEMBER);
}

/* process_user_event / process_query_event (snapshot.rs:663-684): the largest ltime
 * handed to the application */
static inline void snap_clock(orc_world* w, uint32_t m, int which, uint64_t ltime) {
  if (!w->snap_sn) return;
  uint64_t* sn = w->snap_sn + (size_t)m * 4;
  if (!(sn[3] & 1) && ltime > sn[which]) sn[which] = ltime;
}

int orc_world_init(orc_world* w, const orc_world_cfg* c) {
  memset(w, 0, sizeof(*w));
  if (c->n < 2 || c->s == 0 || c->s > c->n || c->qcap == 0 || c->qcap > ORC_MAX_QCAP || c->ebuf == 0 ||
      c->qbuf == 0 || c->slot_k == 0 || c->fanout == 0 || c->fanout >= c->n || c->max_refute == 0 ||
      c->cap_rumors == 0 || (c->cap_rumors & (c->cap_rumors - 1)) || c->cap_rumors > (1u << 30))
    return -1;
  w->n = c->n;
  w->s = c->s;
  w->qcap = c->qcap;
  w->ebuf = c->ebuf;
  w->qbuf = c->qbuf;
  w->slot_k = c->slot_k;
  w->fanout = c->fanout;
  w->limit = c->limit;
  w->overhead = c->overhead;
  w->tx_limit = orc_retransmit_limit(c->retransmit_mult, c->n);
  w->max_refute = c->max_refute;
  w->seed = c->seed;
  size_t n = c->n, s = c->s;
#define A(p, cnt) (w->p = calloc((cnt), sizeof(*w->p)), w->p == NULL)
  if (A(clock, n) || A(eclock, n) || A(qclock, n) || A(emin, n) || A(qmin, n) || A(digest, n) ||
      A(alive, n) || A(serf_state, n) || A(err, n) || A(subj_member, s) || A(member_subj, n) ||
      A(refute_cnt, s) || A(refute_ltime, s * c->max_refute) || A(v_ltime, n * s) ||
      A(v_status, n * s) || A(v_kind, n * s) || A(q_rumor, n * 3 * c->qcap) ||
      A(q_seq, n * 3 * c->qcap) || A(q_tx, n * 3 * c->qcap) || A(q_len, n * 3 * c->qcap) ||
      A(q_next_seq, n * 3) || A(eb_ltime, n * c->ebuf) || A(eb_cnt, n * c->ebuf) ||
      A(eb_keys, n * c->ebuf * c->slot_k) || A(qb_ltime, n * c->qbuf) || A(qb_cnt, n * c->qbuf) ||
      A(qb_ids, n * c->qbuf * c->slot_k) || A(rumors, 2 * (size_t)c->cap_rumors) || A(v_time, n * s) ||
      A(q_pruned, n) || A(q_expired, n) || A(q_hwm, n * 3) || A(q_hole, n * 3)) {
    orc_world_free(w);
    return -1;
  }
#undef A
  if (c->max_user_event_size > ORC_USER_EVENT_SIZE_LIMIT || c->query_size_limit > 0xFFFE) { /* base.rs:69-70 */
    orc_world_free(w);
    return -1;
  }
  w->max_ue = c->max_user_event_size ? c->max_user_event_size : 512;
  w->query_limit = c->query_size_limit ? c->query_size_limit : 1024;
  for (int q = 0; q < 3; ++q) {
    if (c->qdepth[q] > c->qcap) {
      orc_world_free(w);
      return -1;
    }
    w->qd[q] = c->qdepth[q] ? c->qdepth[q] : c->qcap;
  }
  w->cap_rumors = c->cap_rumors;
  w->rbits = 0;
  while ((1u << w->rbits) < c->cap_rumors) w->rbits++;
  for (size_t m = 0; m < n; ++m) {
    /* Serf::new: every clock incremented once (base.rs:195-199) */
    w->clock[m] = 1;
    w->eclock[m] = 1;
    w->qclock[m] = 1;
    w->alive[m] = 1;
    w->serf_state[m] = ORC_SERF_ALIVE;
    w->member_subj[m] = -1;
  }
  for (size_t i = 0; i < n * 3 * c->qcap; ++i) w->q_rumor[i] = EMPTY_RUMOR;
  return 0;
}

void orc_world_free(orc_world* w) {
  void* ptrs[] = {w->clock, w->eclock, w->qclock, w->emin, w->qmin, w->digest, w->alive,
                  w->serf_state, w->err, w->subj_member, w->member_subj, w->refute_cnt,
                  w->refute_ltime, w->v_ltime, w->v_status, w->v_kind, w->q_rumor, w->q_seq,
                  w->q_tx, w->q_len, w->q_next_seq, w->eb_ltime, w->eb_cnt, w->eb_keys,
                  w->qb_ltime, w->qb_cnt, w->qb_ids, w->rumors, w->v_time, w->q_pruned, w->q_expired,
                  w->dlog, w->dcnt, w->snap_bits, w->snap_sn, w->q_hwm, w->act_status, w->q_hole};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i) free(ptrs[i]);
  memset(w, 0, sizeof(*w));
}

/* upsert_intent  base.rs:1797-1828 (recent_intents: one entry per unknown node) */
int orc_upsert_intent(orc_world* w, uint32_t m, uint32_t subj, uint8_t kind, uint64_t ltime) {
  size_t e = (size_t)m * w->s + subj;
  if (w->v_kind[e] == ORC_K_UNKNOWN) {
    w->v_kind[e] = kind;
    w->v_ltime[e] = ltime;
    w->v_time[e] = w->now; /* wall_time: stamper() */
    return 1;
  }
  if (ltime > w->v_ltime[e]) {
    w->v_kind[e] = kind;
    w->v_ltime[e] = ltime;
    w->v_time[e] = w->now;
    return 1;
  }
  return 0;
}

/* handle_node_join_intent  base.rs:1302-1337 */
int orc_handle_join_intent(orc_world* w, uint32_t m, uint32_t subj, uint64_t ltime) {
  orc_clock_witness(&w->clock[m], ltime);
  size_t e = (size_t)m * w->s + subj;
  if (w->v_kind[e] == ORC_K_KNOWN) {
    if (ltime <= w->v_ltime[e]) return 0;
    w->v_ltime[e] = ltime;
    if (w->v_status[e] == ORC_ST_LEAVING) w->v_status[e] = ORC_ST_ALIVE;
    return ORC_F_REBROADCAST;
  }
  return orc_upsert_intent(w, m, subj, ORC_K_INTENT_JOIN, ltime) ? ORC_F_REBROADCAST : 0;
}

static void erase_entry(orc_world* w, size_t e);
static void snap_leave(orc_world* w, uint32_t m);

/* handle_prune  base.rs:1587-1612: erase_node! (members.states.remove; the member also
 * leaves left_members) and a Reap MemberEvent.  The reference first sleeps
 * broadcast_timeout + leave_propagate_delay when the member is Leaving; the round
 * model erases at once. */
static int handle_prune(orc_world* w, uint32_t m, uint32_t subj, size_t e) {
  erase_entry(w, e);
  digest_member_event(w, m, EV_REAP, subj);
  return ORC_F_PRUNE;
}

/* handle_node_leave_intent  base.rs:1409-1528 */
int orc_handle_leave_intent(orc_world* w, uint32_t m, uint32_t subj, uint64_t ltime, int prune,
                            uint64_t* refute_ltime) {
  uint8_t state = w->serf_state[m]; /* base.rs:1410 */
  orc_clock_witness(&w->clock[m], ltime);
  size_t e = (size_t)m * w->s + subj;
  if (w->v_kind[e] != ORC_K_KNOWN)
    return orc_upsert_intent(w, m, subj, ORC_K_INTENT_LEAVE, ltime) ? ORC_F_REBROADCAST : 0;
  if (ltime <= w->v_ltime[e]) return 0;
  if (w->member_subj[m] == (int32_t)subj && state == ORC_SERF_ALIVE) { /* refute (1437-1447) */
    if (refute_ltime) *refute_ltime = w->clock[m];
    return ORC_F_REFUTE;
  }
  w->v_ltime[e] = ltime; /* 1464 */
  switch (w->v_status[e]) {
    case ORC_ST_NONE: return 0;
    case ORC_ST_ALIVE: /* 1469-1478 */
      w->v_status[e] = ORC_ST_LEAVING;
      return ORC_F_REBROADCAST | (prune ? handle_prune(w, m, subj, e) : 0);
    case ORC_ST_LEAVING:
    case ORC_ST_LEFT: /* 1479-1486 */
      return ORC_F_REBROADCAST | (prune ? handle_prune(w, m, subj, e) : 0);
    case ORC_ST_FAILED: /* 1487-1526: Failed -> Left, Leave event, then the prune */
      w->v_status[e] = ORC_ST_LEFT;
      digest_member_event(w, m, EV_LEAVE, subj);
      return ORC_F_REBROADCAST | ORC_F_MEMBER_EVENT | (prune ? handle_prune(w, m, subj, e) : 0);
    default: return 0;
  }
}

/* handle_node_join (memberlist NotifyJoin)  base.rs:1167-1298 */
int orc_handle_node_join(orc_world* w, uint32_t m, uint32_t subj) {
  size_t e = (size_t)m * w->s + subj;
  w->v_time[e] = 0; /* leave_time: None (1226, 1265) */
  if (w->v_kind[e] == ORC_K_KNOWN) {
    w->v_status[e] = ORC_ST_ALIVE; /* status_time kept (1225) */
  } else {
    uint8_t status = ORC_ST_ALIVE;
    uint64_t st = 0;
    if (w->v_kind[e] == ORC_K_INTENT_JOIN) st = w->v_ltime[e];
    if (w->v_kind[e] == ORC_K_INTENT_LEAVE) {
      st = w->v_ltime[e];
      status = ORC_ST_LEAVING;
    }
    w->v_kind[e] = ORC_K_KNOWN;
    w->v_status[e] = status;
    w->v_ltime[e] = st;
  }
  digest_member_event(w, m, EV_JOIN, subj);
  return ORC_F_MEMBER_EVENT;
}

/* handle_node_update (memberlist NotifyUpdate)  base.rs:1532-1583: a member with state
 * gets its attributes (tags: host-side) and the Update MemberEvent */
int orc_handle_node_update(orc_world* w, uint32_t m, uint32_t subj) {
  if (w->v_kind[(size_t)m * w->s + subj] != ORC_K_KNOWN) return 0;
  digest_member_event(w, m, EV_UPDATE, subj);
  return ORC_F_MEMBER_EVENT;
}

/* handle_node_leave (memberlist NotifyLeave)  base.rs:1339-1407 */
int orc_handle_node_leave(orc_world* w, uint32_t m, uint32_t subj) {
  size_t e = (size_t)m * w->s + subj;
  if (w->v_kind[e] != ORC_K_KNOWN) return 0;
  if (w->v_status[e] == ORC_ST_LEAVING) {
    w->v_status[e] = ORC_ST_LEFT;
    w->v_time[e] = w->now; /* leave_time = now (1355) */
    digest_member_event(w, m, EV_LEAVE, subj);
  } else if (w->v_status[e] == ORC_ST_ALIVE) {
    w->v_status[e] = ORC_ST_FAILED;
    w->v_time[e] = w->now; /* (1364) */
    digest_member_event(w, m, EV_FAILED, subj);
  } else {
    return 0;
  }
  return ORC_F_MEMBER_EVENT;
}

int orc_world_set_delivery_log(orc_world* w, uint32_t per_member) {
  free(w->dlog);
  free(w->dcnt);
  w->dlog = NULL;
  w->dcnt = NULL;
  w->dcap = 0;
  if (!per_member) return 0;
  w->dlog = (uint64_t*)calloc((size_t)w->n * per_member * 3, sizeof(uint64_t));
  w->dcnt = (uint32_t*)calloc(w->n, sizeof(uint32_t));
  if (!w->dlog || !w->dcnt) return -1;
  w->dcap = per_member;
  return 0;
}

/* event_tx.send(UserEvent) (base.rs:831-835) into the member's delivery log */
static void dlog_put(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key, uint64_t flags) {
  if (!w->dcap) return;
  uint32_t k = w->dcnt[m];
  if (k < w->dcap) {
    uint64_t* e = w->dlog + ((size_t)m * w->dcap + k) * 3;
    e[0] = ltime;
    e[1] = key;
    e[2] = flags; /* a word of its own: a user event's ltime is a full u64 off the wire */
  } else {
    w->err[m] |= ORC_E_DLOG;
  }
  w->dcnt[m] = k + 1;
}

int orc_handle_user_event(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key) {
  return orc_handle_user_event_cc(w, m, ltime, key, 0);
}

/* handle_user_event  base.rs:770-837 */
int orc_handle_user_event_cc(orc_world* w, uint32_t m, uint64_t ltime, uint64_t key, int cc) {
  orc_clock_witness(&w->eclock[m], ltime);
  if (ltime < w->emin[m]) return 0;
  uint64_t B = w->ebuf, cur = w->eclock[m];
  if (cur > B && ltime < cur - B) return 0;
  size_t slot = (size_t)m * w->ebuf + (size_t)(ltime % B);
  uint64_t* keys = w->eb_keys + slot * w->slot_k;
  if (w->eb_cnt[slot]) {
    for (uint32_t i = 0; i < w->eb_cnt[slot]; ++i)
      if (keys[i] == key) return 0;
    if (w->eb_cnt[slot] < w->slot_k) keys[w->eb_cnt[slot]++] = key;
    else w->err[m] |= ORC_E_EVSLOT_FULL;
  } else {
    w->eb_ltime[slot] = ltime;
    keys[0] = key;
    w->eb_cnt[slot] = 1;
  }
  w->digest[m] = orc_digest_mix(orc_digest_mix(w->digest[m], DIG_USER ^ key), ltime);
  dlog_put(w, m, ltime, key, cc ? ORC_LOG_CC : 0);
  snap_clock(w, m, 0, ltime);
  return ORC_F_REBROADCAST | ORC_F_DELIVER;
}

/* handle_query  base.rs:981-1119 (dedup + rebroadcast decision; filters pass) */
int orc_handle_query(orc_world* w, uint32_t m, uint64_t ltime, uint32_t id, int no_broadcast) {
  orc_clock_witness(&w->qclock[m], ltime);
  if (ltime < w->qmin[m]) return 0;
  uint64_t cur = w->qclock[m], B = w->qbuf;
  if (cur > B && B < cur - B) return 0; /* reference quirk base.rs:999 */
  size_t slot = (size_t)m * w->qbuf + (size_t)(ltime % B);
  uint32_t* ids = w->qb_ids + slot * w->slot_k;
  if (w->qb_cnt[slot]) {
    if (w->qb_ltime[slot] == ltime)
      for (uint32_t i = 0; i < w->qb_cnt[slot]; ++i)
        if (ids[i] == id) return 0;
    if (w->qb_cnt[slot] < w->slot_k) ids[w->qb_cnt[slot]++] = id;
    else w->err[m] |= ORC_E_QSLOT_FULL;
  } else {
    w->qb_ltime[slot] = ltime;
    ids[0] = id;
    w->qb_cnt[slot] = 1;
  }
  w->digest[m] = orc_digest_mix(orc_digest_mix(w->digest[m], DIG_QUERY ^ id), ltime);
  snap_clock(w, m, 1, ltime);
  return (no_broadcast ? 0 : ORC_F_REBROADCAST) | ORC_F_DELIVER;
}

/* ---- TransmitLimitedQueue model (memberlist; un-vendored, parity unpinned) */
static inline uint64_t tlq_key(uint16_t tx, uint16_t len, uint32_t seq) {
  return ((uint64_t)tx << 48) | ((uint64_t)(0xFFFFu - len) << 32) | (uint64_t)(0xFFFFFFFFu - seq);
}

/* Slot order is free (the queue's CONTENT is what the model defines): a queue's live items
 * sit in slots [0, hwm), so every scan stops at the high-water mark. */
void orc_queue_insert(orc_world* w, uint32_t m, uint32_t q, uint32_t rumor) {
  size_t base = ((size_t)m * 3 + q) * w->qcap;
  uint32_t* hwm = &w->q_hwm[(size_t)m * 3 + q];
  uint32_t* hole = &w->q_hole[(size_t)m * 3 + q];
  uint32_t seq = w->q_next_seq[(size_t)m * 3 + q]++;
  uint16_t len = w->rumors[orc_rumor_index(w, rumor)].msg_len;
  uint32_t slot = EMPTY_RUMOR;
  /* the first free slot (no slot below *hole is free) */
  for (uint32_t i = *hole; i < *hwm; ++i)
    if (w->q_rumor[base + i] == EMPTY_RUMOR) {
      slot = i;
      break;
    }
  if (slot == EMPTY_RUMOR && *hwm < w->qd[q]) slot = (*hwm)++;
  if (slot != EMPTY_RUMOR) *hole = slot + 1;
  if (slot == EMPTY_RUMOR) { /* full: prune the last item in send order */
    w->q_pruned[m]++;
    w->err[m] |= ORC_E_QUEUE_PRUNE;
    uint64_t kmax = 0;
    for (uint32_t i = 0; i < *hwm; ++i) {
      uint64_t k = tlq_key(w->q_tx[base + i], w->q_len[base + i], w->q_seq[base + i]);
      if (slot == EMPTY_RUMOR || k > kmax) {
        kmax = k;
        slot = i;
      }
    }
    if (tlq_key(0, len, seq) > kmax) return; /* the new item itself is pruned */
  }
  w->q_rumor[base + slot] = rumor;
  w->q_seq[base + slot] = seq;
  w->q_tx[base + slot] = 0;
  w->q_len[base + slot] = len;
}

uint32_t orc_rumor_generations(const orc_world* w) {
  /* even, so the parity alternates across the wrap; ids gen << rbits | slot never reach
   * 0xFFFFFFFF (the empty-queue-slot marker) */
  return (uint32_t)((1ull << (32 - w->rbits)) - 2);
}

uint32_t orc_rumor_index(const orc_world* w, uint32_t rid) {
  /* two generations resident: the id's generation parity selects the table half */
  return rid & ((w->cap_rumors << 1) - 1);
}

int orc_rumor_live(const orc_world* w, uint32_t rid) {
  const uint32_t G = orc_rumor_generations(w);
  return (w->gen + G - (rid >> w->rbits) % G) % G < 2;
}

uint32_t orc_queue_expire(orc_world* w, uint32_t m, uint32_t q) {
  size_t base = ((size_t)m * 3 + q) * w->qcap;
  uint32_t cnt = 0;
  const uint32_t hwm = w->q_hwm[(size_t)m * 3 + q];
  for (uint32_t i = 0; i < hwm; ++i) {
    if (w->q_rumor[base + i] == EMPTY_RUMOR || orc_rumor_live(w, w->q_rumor[base + i])) continue;
    w->q_rumor[base + i] = EMPTY_RUMOR;
    w->q_seq[base + i] = 0;
    w->q_tx[base + i] = 0;
    w->q_len[base + i] = 0;
    if (i < w->q_hole[(size_t)m * 3 + q]) w->q_hole[(size_t)m * 3 + q] = i;
    cnt++;
  }
  return cnt;
}

/* get_broadcasts: lowest transmits first, then the largest message that fits,
 * then the newest; picked items are re-inserted with transmits+1 or retired
 * at the retransmit limit (memberlist queue.go GetBroadcasts, restated). */
uint32_t orc_queue_get_broadcasts(orc_world* w, uint32_t m, uint32_t q, uint32_t limit,
                                  uint32_t* out, uint32_t max_out, uint32_t* bytes_used) {
  size_t base = ((size_t)m * 3 + q) * w->qcap;
  const uint32_t hwm = w->q_hwm[(size_t)m * 3 + q];
  int64_t used = 0;
  uint32_t cnt = 0;
  /* The live items' keys are gathered once (the oracle's speed only); each pick is then the
   * smallest key among the unpicked items that fit the budget left (keys are distinct: seq is
   * unique in a queue).  A picked item's key becomes UINT64_MAX. */
  uint64_t kk[ORC_MAX_QCAP];
  uint32_t ki[ORC_MAX_QCAP];
  uint32_t picked[ORC_MAX_QCAP];
  uint32_t kn = 0, np = 0;
  for (uint32_t i = 0; i < hwm; ++i) {
    if (w->q_rumor[base + i] == EMPTY_RUMOR) continue;
    kk[kn] = tlq_key(w->q_tx[base + i], w->q_len[base + i], w->q_seq[base + i]);
    ki[kn++] = i;
  }
  for (;;) {
    int64_t free_b = (int64_t)limit - used - (int64_t)w->overhead;
    if (free_b <= 0) break;
    uint32_t best = EMPTY_RUMOR;
    uint64_t kbest = UINT64_MAX;
    for (uint32_t j = 0; j < kn; ++j) {
      if (kk[j] >= kbest) continue;
      /* the key's length field: 0xFFFF - len */
      if ((int64_t)(0xFFFFu - (uint32_t)((kk[j] >> 32) & 0xFFFFu)) > free_b) continue;
      kbest = kk[j];
      best = j;
    }
    if (best == EMPTY_RUMOR) break;
    const uint32_t i = ki[best];
    kk[best] = UINT64_MAX;
    if (cnt < max_out) out[cnt] = w->q_rumor[base + i];
    cnt++;
    used += (int64_t)w->overhead + w->q_len[base + i];
    picked[np++] = i;
  }
  for (uint32_t j = 0; j < np; ++j) {
    const uint32_t i = picked[j];
    if ((uint32_t)w->q_tx[base + i] + 1 >= w->tx_limit) {
      w->q_rumor[base + i] = EMPTY_RUMOR;
      if (i < w->q_hole[(size_t)m * 3 + q]) w->q_hole[(size_t)m * 3 + q] = i;
    } else {
      w->q_tx[base + i]++;
    }
  }
  *bytes_used = (uint32_t)used;
  return cnt;
}

/* members.states.len() of member m (the map holds every member the node knows):
 * the n - s untracked members (implicitly Alive; the local node is one of them unless
 * it is a subject), the local node if it is a subject, and the tracked subjects whose
 * entry is KNOWN (left / failed members stay in the map until reaped, base.rs:519-573) */
uint64_t orc_states_len(const orc_world* w, uint32_t m) {
  const size_t row = (size_t)m * w->s;
  uint64_t known = (uint64_t)(w->n - w->s) + (w->member_subj[m] >= 0 ? 1u : 0u);
  for (uint32_t subj = 0; subj < w->s; ++subj)
    if ((int32_t)subj != w->member_subj[m] && w->v_kind[row + subj] == ORC_K_KNOWN) known++;
  return known;
}

static int u64_cmp(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

void orc_check_queues_phase(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth,
                            uint32_t depth_warning, uint32_t period, uint32_t phase, uint64_t* stats) {
  uint64_t st[9] = {0};
  uint64_t* keys = NULL;
  size_t kcap = 0;
  if (!period) period = 1;
  for (uint32_t m = 0; m < w->n; ++m) {
    if (m % period != phase) continue; /* this node's checker is not due this round */
    /* get_queue_max  base.rs:748-759: each node's checker reads its own members.states */
    uint64_t mx = max_queue_depth;
    if (min_queue_depth > 0) {
      mx = 2ull * orc_states_len(w, m);
      if (mx < min_queue_depth) mx = min_queue_depth;
    }
    for (uint32_t q = 0; q < 3; ++q) {
      size_t base = ((size_t)m * 3 + q) * w->qcap;
      const uint32_t hwm = w->q_hwm[(size_t)m * 3 + q];
      uint32_t numq = 0;
      for (uint32_t i = 0; i < hwm; ++i) numq += w->q_rumor[base + i] != EMPTY_RUMOR;
      st[q] += numq;
      if (numq >= depth_warning) st[3 + q]++;
      if (numq <= mx) continue;
      /* numq >= max -> prune(max): the items past the max-th in send order go, the largest
       * first (the keys are distinct: seq is unique within a queue), so the max smallest stay */
      if (numq > kcap) {
        kcap = numq;
        keys = (uint64_t*)realloc(keys, kcap * sizeof(uint64_t));
      }
      uint32_t k = 0;
      for (uint32_t i = 0; i < hwm; ++i)
        if (w->q_rumor[base + i] != EMPTY_RUMOR) keys[k++] = tlq_key(w->q_tx[base + i], w->q_len[base + i], w->q_seq[base + i]);
      qsort(keys, k, sizeof(uint64_t), u64_cmp);
      const uint64_t T = mx ? keys[mx - 1] : 0;
      for (uint32_t i = 0; i < hwm; ++i) {
        if (w->q_rumor[base + i] == EMPTY_RUMOR) continue;
        if (mx && tlq_key(w->q_tx[base + i], w->q_len[base + i], w->q_seq[base + i]) <= T) continue;
        if (i < w->q_hole[(size_t)m * 3 + q]) w->q_hole[(size_t)m * 3 + q] = i;
        w->q_rumor[base + i] = EMPTY_RUMOR;
        w->q_seq[base + i] = 0;
        w->q_tx[base + i] = 0;
        w->q_len[base + i] = 0;
      }
      st[6 + q] += numq - mx;
    }
  }
  free(keys);
  if (stats) memcpy(stats, st, sizeof(st));
}

void orc_check_queues(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                      uint64_t* stats) {
  orc_check_queues_phase(w, max_queue_depth, min_queue_depth, depth_warning, 1, 0, stats);
}

void orc_world_set_checker(orc_world* w, uint32_t max_queue_depth, uint32_t min_queue_depth, uint32_t depth_warning,
                           uint32_t period) {
  w->chk_period = period;
  w->chk_max = max_queue_depth;
  w->chk_min = min_queue_depth;
  w->chk_warn = depth_warning;
  memset(w->chk_stats, 0, sizeof(w->chk_stats));
}

/* kRandomNodes model: k distinct live peers != m, Philox-drawn (memberlist util.go; unpinned) */
uint32_t orc_pick_peers(uint64_t seed, uint32_t n, const uint8_t* alive, uint32_t m, uint32_t round,
                        uint32_t k, uint32_t* out) {
  uint32_t key[2];
  seed_key(seed, key);
  uint32_t cnt = 0;
  for (uint32_t a = 0; a < 64 * k && cnt < k; ++a) {
    uint32_t ctr[4] = {a, PURPOSE_PEER << 24, m, round}, o[4];
    orc_philox4x32(ctr, key, o);
    uint32_t p = mulhi32(o[0], n - 1);
    if (p >= m) p++;
    if (!alive[p]) continue;
    int dup = 0;
    for (uint32_t j = 0; j < cnt; ++j) dup |= (out[j] == p);
    if (dup) continue;
    out[cnt++] = p;
  }
  return cnt;
}

static uint32_t queue_of(uint8_t type) {
  return type == ORC_MSG_USER_EVENT ? ORC_Q_EVENT : (type == ORC_MSG_QUERY ? ORC_Q_QUERY : ORC_Q_INTENT);
}

static uint32_t new_rumor(orc_world* w, uint32_t id, uint8_t type, uint8_t flags, uint32_t subject,
                          uint64_t ltime, uint64_t key, uint32_t name_len, uint32_t payload_len) {
  orc_rumor* r = &w->rumors[orc_rumor_index(w, id)];
  r->type = type;
  r->flags = flags;
  r->subject = subject;
  r->ltime = ltime;
  r->key = key;
  r->msg_len = (uint16_t)orc_msg_len(type, ltime, name_len, payload_len);
  return id;
}

static void push_refute(orc_world* w, uint32_t m, uint64_t ltime) {
  int32_t s = w->member_subj[m];
  if (s < 0) return;
  if (w->refute_cnt[s] < w->max_refute) w->refute_ltime[(size_t)s * w->max_refute + w->refute_cnt[s]++] = ltime;
  else w->err[m] |= ORC_E_REFUTE_FULL;
}

/* apply one received rumor at receiver r  (notify_message, delegate.rs:157-305) */
static void merge_one(orc_world* w, uint32_t r, uint32_t rid) {
  const orc_rumor* ru = &w->rumors[orc_rumor_index(w, rid)];
  int f = 0;
  uint64_t refute = 0;
  switch (ru->type) {
    case ORC_MSG_JOIN: f = orc_handle_join_intent(w, r, ru->subject, ru->ltime); break;
    case ORC_MSG_LEAVE:
      f = orc_handle_leave_intent(w, r, ru->subject, ru->ltime, ru->flags & 1, &refute);
      break;
    case ORC_MSG_USER_EVENT: f = orc_handle_user_event_cc(w, r, ru->ltime, ru->key, ru->flags & 1); break;
    case ORC_MSG_QUERY: f = orc_handle_query(w, r, ru->ltime, (uint32_t)ru->key, ru->flags & 1); break;
    default: return;
  }
  if (f & ORC_F_REFUTE) push_refute(w, r, refute);
  if (f & ORC_F_REBROADCAST) orc_queue_insert(w, r, queue_of(ru->type), rid);
}

/* broadcast_join  base.rs:396-412 */
static void broadcast_join(orc_world* w, uint32_t m, uint64_t ltime, uint32_t rid) {
  int32_t subj = w->member_subj[m];
  orc_clock_witness(&w->clock[m], ltime);
  orc_handle_join_intent(w, m, (uint32_t)subj, ltime);
  new_rumor(w, rid, ORC_MSG_JOIN, 0, (uint32_t)subj, ltime, 0, 0, 0);
  orc_queue_insert(w, m, ORC_Q_INTENT, rid);
}

/* ---- the round's member-parallel phases.  Members are independent inside each
 * phase (a handler touches only its receiver's state; the rumor table and the
 * liveness array are read-only there), so the threaded round is identical to
 * the sequential one: it only partitions the member loops over threads. */
typedef struct {
  orc_world* w;
  uint32_t lo, hi, round;
  const orc_ml_event* ml;
  uint32_t n_ml;
  /* emission output (sender range [lo, hi) in sender order) */
  uint32_t *rec_recv, *rec_rumor;
  size_t nrec, cap;
  /* merge input */
  const uint32_t *off, *order;
  uint64_t merges, sends;
  int phase, fail;
} world_job;

/* 1. memberlist-detected transitions (M6) at every live member but the subject.
 *    Per member: events in order; its liveness changes only by events about itself. */
static void phase_ml(world_job* j) {
  orc_world* w = j->w;
  for (uint32_t m = j->lo; m < j->hi; ++m) {
    uint8_t al = w->alive[m];
    for (uint32_t e = 0; e < j->n_ml; ++e) {
      uint32_t subj = j->ml[e].subject, sm = w->subj_member[subj];
      if (sm == m && j->ml[e].set_alive == 1) {
        al = 1;
        w->serf_state[m] = ORC_SERF_ALIVE;
      }
      if (al && m != sm) {
        if (j->ml[e].kind == ORC_ML_JOIN) orc_handle_node_join(w, m, subj);
        else if (j->ml[e].kind == ORC_ML_UPDATE) orc_handle_node_update(w, m, subj);
        else orc_handle_node_leave(w, m, subj);
      }
      if (sm == m && j->ml[e].set_alive == 0) al = 0;
    }
    w->alive[m] = al;
  }
}

/* 4. emission: each live sender, k peers, broadcast_messages (delegate.rs:307-374) */
static void phase_emit(world_job* j) {
  orc_world* w = j->w;
  /* records per (sender, peer): every message costs at least overhead + 15 B of the budget
   * (the shortest of the length model, orc_msg_len), so this bounds one peer's picks */
  const uint32_t per_peer = w->limit / (w->overhead + 15) + 1;
  const uint32_t n = w->n, k = w->fanout, cap_t = 3 * w->qcap < per_peer ? 3 * w->qcap : per_peer;
  uint32_t peers[64], buf[3 * ORC_MAX_QCAP];
  j->cap = (size_t)(j->hi - j->lo) * k * cap_t;
  j->rec_recv = (uint32_t*)malloc((j->cap ? j->cap : 1) * sizeof(uint32_t));
  j->rec_rumor = (uint32_t*)malloc((j->cap ? j->cap : 1) * sizeof(uint32_t));
  if (!j->rec_recv || !j->rec_rumor) {
    j->fail = 1;
    return;
  }
  for (uint32_t m = j->lo; m < j->hi; ++m) {
    if (!w->alive[m]) continue;
    uint32_t np = orc_pick_peers(w->seed, n, w->alive, m, j->round, k, peers);
    for (uint32_t p = 0; p < np; ++p) {
      uint32_t used = 0, got = 0, b;
      for (uint32_t q = 0; q < 3; ++q) {
        got += orc_queue_get_broadcasts(w, m, q, w->limit - used, buf + got, cap_t - got, &b);
        used += b;
      }
      for (uint32_t i = 0; i < got; ++i) {
        j->rec_recv[j->nrec] = peers[p];
        j->rec_rumor[j->nrec] = buf[i];
        j->nrec++;
      }
      j->sends += got;
    }
  }
}

/* 5. merge at every live receiver, its records in canonical (sender, position) order */
static void phase_merge(world_job* j) {
  orc_world* w = j->w;
  for (uint32_t r = j->lo; r < j->hi; ++r) {
    if (!w->alive[r]) continue;
    for (uint32_t i = j->off[r]; i < j->off[r + 1]; ++i) {
      merge_one(w, r, j->order[i]);
      j->merges++;
    }
  }
}

static void* world_worker(void* arg) {
  world_job* j = (world_job*)arg;
  if (j->phase == 1) phase_ml(j);
  else if (j->phase == 4) phase_emit(j);
  else phase_merge(j);
  return NULL;
}

static void run_phase(world_job* jobs, int nt) {
  if (nt == 1) {
    world_worker(&jobs[0]);
    return;
  }
  pthread_t th[256];
  for (int i = 0; i < nt; ++i) pthread_create(&th[i], NULL, world_worker, &jobs[i]);
  for (int i = 0; i < nt; ++i) pthread_join(th[i], NULL);
}

int orc_world_round_mt(orc_world* w, uint32_t round, const orc_ml_event* ml, uint32_t n_ml,
                       const orc_action* acts, uint32_t n_acts, int nthreads) {
  const uint32_t n = w->n;
  int nt = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
  if ((uint32_t)nt > n) nt = (int)n;
  world_job jobs[256];
  memset(jobs, 0, sizeof(world_job) * (size_t)nt);
  const uint32_t per = (n + (uint32_t)nt - 1) / (uint32_t)nt;
  for (int i = 0; i < nt; ++i) {
    uint32_t lo = (uint32_t)i * per, hi = lo + per;
    jobs[i].w = w;
    jobs[i].lo = lo < n ? lo : n;
    jobs[i].hi = hi < n ? hi : n;
    jobs[i].round = round;
    jobs[i].ml = ml;
    jobs[i].n_ml = n_ml;
  }
  w->now = round;
  /* rumor ids of this round: [refutes: s*max_refute][actions: n_acts], a contiguous
   * block of the ring (restarting at slot 0 with the next generation when it would
   * cross the end); id = generation << rbits | slot */
  uint32_t need = w->s * w->max_refute + n_acts;
  if (need > w->cap_rumors) return -1;
  if (w->n_rumors + need > w->cap_rumors) {
    w->n_rumors = 0;
    w->gen = (w->gen + 1) % orc_rumor_generations(w);
    /* this generation reuses the table half of generation gen - 2: its queued ids expire */
    for (uint32_t m = 0; m < n; ++m)
      for (uint32_t q = 0; q < 3; ++q) w->q_expired[m] += orc_queue_expire(w, m, q);
  }
  const uint32_t slot0 = w->n_rumors;
  uint32_t base = (uint32_t)(((uint64_t)w->gen << w->rbits) | slot0);
  for (uint32_t i = 0; i < need; ++i) w->rumors[orc_rumor_index(w, base + i)].type = 0xFF;
  w->n_rumors += need;
  if (w->dcap) memset(w->dcnt, 0, (size_t)n * sizeof(uint32_t)); /* the round's delivery log */

  /* 1. memberlist transitions */
  if (n_ml) {
    for (int i = 0; i < nt; ++i) jobs[i].phase = 1;
    run_phase(jobs, nt);
  }

  /* 2. refutations scheduled by the previous round's merges (spawn_detach) */
  for (uint32_t s = 0; s < w->s; ++s) {
    uint32_t m = w->subj_member[s];
    for (uint32_t i = 0; i < w->refute_cnt[s]; ++i)
      if (w->alive[m]) broadcast_join(w, m, w->refute_ltime[(size_t)s * w->max_refute + i],
                                      base + s * w->max_refute + i);
    w->refute_cnt[s] = 0;
  }

  /* 3. originations (api.rs / base.rs entry points) */
  uint32_t abase = base + w->s * w->max_refute;
  if (n_acts > w->act_cap) {
    int32_t* p = (int32_t*)realloc(w->act_status, (size_t)n_acts * sizeof(int32_t));
    if (!p) return -1;
    w->act_status = p;
    w->act_cap = n_acts;
  }
  w->last_n_acts = n_acts;
  for (uint32_t a = 0; a < n_acts; ++a) {
    const orc_action* x = &acts[a];
    uint32_t m = x->member, rid = abase + a;
    if (!w->alive[m]) {
      w->act_status[a] = ORC_SKIPPED;
      continue;
    }
    /* the size checks return before anything moves (api.rs:255-287; base.rs:919-921) */
    int32_t st = 0;
    if (x->act == ORC_ACT_USER_EVENT) st = orc_user_event_check(w->max_ue, w->eclock[m], x->name_len, x->payload_len);
    if (x->act == ORC_ACT_QUERY) st = orc_query_check(w->query_limit, w->qclock[m], x->name_len, x->payload_len);
    w->act_status[a] = st;
    if (st) continue;
    switch (x->act) {
      case ORC_ACT_JOIN_SELF: /* Serf::join -> broadcast_join(clock.time()) */
        w->serf_state[m] = ORC_SERF_ALIVE;
        broadcast_join(w, m, w->clock[m], rid);
        break;
      case ORC_ACT_LEAVE_SELF: { /* Serf::leave  api.rs:473-503 */
        w->serf_state[m] = ORC_SERF_LEAVING;
        uint64_t lt = w->clock[m];
        if (w->snap_sn) snap_leave(w, m);
        orc_clock_increment(&w->clock[m]);
        uint32_t subj = (uint32_t)w->member_subj[m];
        orc_handle_leave_intent(w, m, subj, lt, 0, NULL);
        new_rumor(w, rid, ORC_MSG_LEAVE, 0, subj, lt, 0, 0, 0);
        orc_queue_insert(w, m, ORC_Q_INTENT, rid);
        break;
      }
      case ORC_ACT_FORCE_LEAVE: { /* force_leave  base.rs:474-500 */
        uint64_t lt = w->clock[m], ref = 0;
        int f = orc_handle_leave_intent(w, m, x->subject, lt, x->flags & 1, &ref);
        if (f & ORC_F_REFUTE) push_refute(w, m, ref);
        new_rumor(w, rid, ORC_MSG_LEAVE, (uint8_t)(x->flags & 1), x->subject, lt, 0, 0, 0);
        orc_queue_insert(w, m, ORC_Q_INTENT, rid);
        break;
      }
      case ORC_ACT_USER_EVENT: { /* Serf::user_event  api.rs:247-315 */
        uint64_t lt = w->eclock[m];
        orc_clock_increment(&w->eclock[m]);
        orc_handle_user_event_cc(w, m, lt, x->key, x->flags & 1);
        new_rumor(w, rid, ORC_MSG_USER_EVENT, (uint8_t)(x->flags & 1), 0, lt, x->key, x->name_len, x->payload_len);
        orc_queue_insert(w, m, ORC_Q_EVENT, rid);
        break;
      }
      case ORC_ACT_QUERY: { /* query_in  base.rs:869-953 */
        uint64_t lt = w->qclock[m];
        orc_handle_query(w, m, lt, (uint32_t)x->key, x->flags & 1);
        new_rumor(w, rid, ORC_MSG_QUERY, (uint8_t)(x->flags & 1), 0, lt, (uint32_t)x->key,
                  x->name_len, x->payload_len);
        orc_queue_insert(w, m, ORC_Q_QUERY, rid);
        break;
      }
      default: break;
    }
  }

  /* 4. emission, sender ranges in parallel; the records stay in sender order */
  for (int i = 0; i < nt; ++i) jobs[i].phase = 4;
  run_phase(jobs, nt);
  int fail = 0;
  size_t nrec = 0;
  for (int i = 0; i < nt; ++i) {
    fail |= jobs[i].fail;
    nrec += jobs[i].nrec;
    w->sends += jobs[i].sends;
  }

  /* 4b. the staggered QueueChecker ticks due this round (each node's checker on its own
   *     timer, base.rs:703-735), between the emission and the merge */
  if (!fail && w->chk_period) {
    uint64_t st[9];
    orc_check_queues_phase(w, w->chk_max, w->chk_min, w->chk_warn, w->chk_period, round % w->chk_period, st);
    for (int i = 0; i < 9; ++i) w->chk_stats[i] += st[i];
  }

  /* 5. merge in canonical (sender, position) order per receiver: stable
   *    counting sort by receiver keeps the sender-major emission order. */
  uint32_t* off = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
  uint32_t* order = (uint32_t*)malloc((nrec ? nrec : 1) * sizeof(uint32_t));
  uint32_t* cur = (uint32_t*)malloc(((size_t)n + 1) * sizeof(uint32_t));
  if (!fail && off && order && cur) {
    for (int t = 0; t < nt; ++t)
      for (size_t i = 0; i < jobs[t].nrec; ++i) off[jobs[t].rec_recv[i] + 1]++;
    for (uint32_t r = 0; r < n; ++r) off[r + 1] += off[r];
    memcpy(cur, off, ((size_t)n + 1) * sizeof(uint32_t));
    for (int t = 0; t < nt; ++t)
      for (size_t i = 0; i < jobs[t].nrec; ++i) order[cur[jobs[t].rec_recv[i]]++] = jobs[t].rec_rumor[i];
    for (int i = 0; i < nt; ++i) {
      jobs[i].phase = 5;
      jobs[i].off = off;
      jobs[i].order = order;
    }
    run_phase(jobs, nt);
    for (int i = 0; i < nt; ++i) w->merges += jobs[i].merges;
  } else {
    fail = 1;
  }
  for (int i = 0; i < nt; ++i) {
    free(jobs[i].rec_recv);
    free(jobs[i].rec_rumor);
  }
  free(off);
  free(order);
  free(cur);
  return fail ? -1 : 0;
}

int orc_world_round(orc_world* w, uint32_t round, const orc_ml_event* ml, uint32_t n_ml,
                    const orc_action* acts, uint32_t n_acts) {
  return orc_world_round_mt(w, round, ml, n_ml, acts, n_acts, 1);
}

/* ------------------------------------------------------------------------ */
/* push/pull anti-entropy  core/src/serf/delegate.rs:422-554                */
int orc_merge_remote_state(orc_world* w, uint32_t r, const orc_pp_state* pp, int is_join, int event_join_ignore) {
  if (!w->alive[r]) return 0;
  /* witness the Lamport clocks first, minus one (delegate.rs:459-475) */
  if (pp->clock > 0) orc_clock_witness(&w->clock[r], pp->clock - 1);
  if (pp->eclock > 0) orc_clock_witness(&w->eclock[r], pp->eclock - 1);
  if (pp->qclock > 0) orc_clock_witness(&w->qclock[r], pp->qclock - 1);
  /* left members first, one past their status time (delegate.rs:477-499) */
  for (uint32_t subj = 0; subj < w->s; ++subj) {
    if (pp->v_kind[subj] != ORC_K_KNOWN || pp->v_status[subj] != ORC_ST_LEFT) continue;
    uint64_t ref = 0;
    int f = orc_handle_leave_intent(w, r, subj, pp->v_ltime[subj] + 1, 0, &ref);
    if (f & ORC_F_REFUTE) push_refute(w, r, ref);
  }
  /* artificial join intents for the other status_ltimes (delegate.rs:501-511) */
  for (uint32_t subj = 0; subj < w->s; ++subj) {
    if (pp->v_kind[subj] != ORC_K_KNOWN || pp->v_status[subj] == ORC_ST_LEFT) continue;
    orc_handle_join_intent(w, r, subj, pp->v_ltime[subj]);
  }
  /* eventJoinIgnore (delegate.rs:513-521) */
  if (is_join && event_join_ignore && pp->eclock > w->emin[r]) w->emin[r] = pp->eclock;
  /* every buffered user event, cc = false (delegate.rs:523-541) */
  for (uint32_t i = 0; i < w->ebuf; ++i)
    for (uint32_t k = 0; k < pp->eb_cnt[i]; ++k)
      orc_handle_user_event(w, r, pp->eb_ltime[i], pp->eb_keys[(size_t)i * w->slot_k + k]);
  return 0;
}

int orc_push_pull(orc_world* w, const uint32_t* recv, const uint32_t* send, uint32_t n, int is_join,
                  int event_join_ignore) {
  const size_t s = w->s, eb = w->ebuf, ek = (size_t)w->ebuf * w->slot_k;
  const size_t per = s * 8 + s + s + eb * 8 + eb * 4 + ek * 8 + 24;
  uint8_t* slab = (uint8_t*)malloc(per * (n ? n : 1));
  orc_pp_state* st = (orc_pp_state*)malloc(sizeof(orc_pp_state) * (n ? n : 1));
  if (!slab || !st) {
    free(slab);
    free(st);
    return -1;
  }
  for (uint32_t i = 0; i < n; ++i) { /* local_state snapshots (delegate.rs:376-420) */
    uint32_t m = send[i];
    uint8_t* p = slab + per * i;
    uint64_t* lt = (uint64_t*)p;
    uint64_t* ebl = lt + s;
    uint64_t* ebk = ebl + eb;
    uint32_t* ebc = (uint32_t*)(ebk + ek);
    uint8_t* stt = (uint8_t*)(ebc + eb);
    uint8_t* kd = stt + s;
    memcpy(lt, w->v_ltime + (size_t)m * s, s * 8);
    memcpy(stt, w->v_status + (size_t)m * s, s);
    memcpy(kd, w->v_kind + (size_t)m * s, s);
    memcpy(ebl, w->eb_ltime + (size_t)m * eb, eb * 8);
    memcpy(ebc, w->eb_cnt + (size_t)m * eb, eb * 4);
    memcpy(ebk, w->eb_keys + (size_t)m * ek, ek * 8);
    st[i] = (orc_pp_state){w->clock[m], w->eclock[m], w->qclock[m], lt, stt, kd, ebl, ebc, ebk};
  }
  for (uint32_t i = 0; i < n; ++i) orc_merge_remote_state(w, recv[i], &st[i], is_join, event_join_ignore);
  free(slab);
  free(st);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Reaper  base.rs:519-601 (reap!, erase_node!), 1782-1784 (reap_intents)   */
static void erase_entry(orc_world* w, size_t e) {
  w->v_kind[e] = ORC_K_UNKNOWN;
  w->v_status[e] = ORC_ST_NONE;
  w->v_ltime[e] = 0;
  w->v_time[e] = 0;
}

int orc_reap(orc_world* w, uint32_t now, uint32_t reconnect_timeout, uint32_t tombstone_timeout,
             uint32_t recent_intent_timeout) {
  for (uint32_t m = 0; m < w->n; ++m) {
    if (!w->alive[m]) continue;
    const size_t row = (size_t)m * w->s;
    /* reap_failed, then reap_left (run(), 588-589) */
    for (int pass = 0; pass < 2; ++pass) {
      const uint8_t st = pass == 0 ? ORC_ST_FAILED : ORC_ST_LEFT;
      const uint32_t timeout = pass == 0 ? reconnect_timeout : tombstone_timeout;
      for (uint32_t subj = 0; subj < w->s; ++subj) {
        size_t e = row + subj;
        if (w->v_kind[e] != ORC_K_KNOWN || w->v_status[e] != st) continue;
        if ((uint32_t)(now - w->v_time[e]) <= timeout) continue; /* leave_time.elapsed() <= timeout */
        erase_entry(w, e);                                        /* members.states.remove */
        digest_member_event(w, m, EV_REAP, subj);                 /* MemberEventType::Reap */
      }
    }
    /* reap_intents: retain (now - wall_time) <= timeout */
    for (uint32_t subj = 0; subj < w->s; ++subj) {
      size_t e = row + subj;
      if (w->v_kind[e] != ORC_K_INTENT_JOIN && w->v_kind[e] != ORC_K_INTENT_LEAVE) continue;
      if ((uint32_t)(now - w->v_time[e]) > recent_intent_timeout) erase_entry(w, e);
    }
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Wire codecs                                                              */
/* byteorder::NetworkEndian */
static void w_u32(uint8_t* d, uint32_t v) {
  for (int i = 3; i >= 0; --i, v >>= 8) d[i] = (uint8_t)v;
}
static uint32_t r_u32(const uint8_t* s) {
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) v = (v << 8) | s[i];
  return v;
}
static void w_f64(uint8_t* d, double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  for (int i = 7; i >= 0; --i, u >>= 8) d[i] = (uint8_t)u;
}
static double r_f64(const uint8_t* s) {
  uint64_t u = 0;
  for (int i = 0; i < 8; ++i) u = (u << 8) | s[i];
  double x;
  memcpy(&x, &u, 8);
  return x;
}

/* transformable::utils::encode_varint / decode_varint (LEB128, at most 10 bytes) */
uint32_t orc_varint_len(uint64_t v) {
  uint32_t n = 1;
  for (; v >= 0x80; v >>= 7) n++;
  return n;
}
uint32_t orc_varint_encode(uint64_t v, uint8_t* dst) {
  uint32_t n = 0;
  for (; v >= 0x80; v >>= 7) dst[n++] = (uint8_t)((v & 0x7F) | 0x80);
  dst[n++] = (uint8_t)v;
  return n;
}
uint32_t orc_varint_decode(const uint8_t* src, uint64_t n, uint64_t* v, int* err) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < 10; ++i) {
    if (i >= n) {
      *err = ORC_E_SHORT;
      return 0;
    }
    if (i == 9 && src[i] > 1) break; /* would overflow u64 */
    x |= (uint64_t)(src[i] & 0x7F) << (7 * i);
    if (!(src[i] & 0x80)) {
      *v = x;
      return i + 1;
    }
  }
  *err = ORC_E_VARINT;
  return 0;
}

/* Coordinate::encode  coordinate.rs:666-692 */
uint32_t orc_coord_encode(const double* row, uint32_t dim, uint8_t* dst) {
  uint32_t encoded_len = 4 + 8 * dim + 8 * 3, off = 0;
  w_u32(dst + off, encoded_len);
  off += 4;
  w_f64(dst + off, row[dim]); /* error */
  off += 8;
  w_f64(dst + off, row[dim + 1]); /* adjustment */
  off += 8;
  w_f64(dst + off, row[dim + 2]); /* height */
  off += 8;
  for (uint32_t i = 0; i < dim; ++i, off += 8) w_f64(dst + off, row[i]);
  return off;
}

/* Coordinate::decode  coordinate.rs:698-745 (release semantics: floor of the portion
 * count; a length below the header would underflow `len - 4 - 3 * 8` and panic) */
int orc_coord_decode(const uint8_t* src, uint64_t src_len, uint32_t max_dim, double* row, uint32_t* dim) {
  if (src_len < 4 + 3 * 8) return ORC_E_SHORT;
  uint64_t len = r_u32(src);
  if (src_len < len) return ORC_E_SHORT;
  if (len < 4 + 3 * 8) return ORC_E_LEN;
  uint64_t num_portion = (len - 4 - 3 * 8) / 8;
  if (num_portion > max_dim) return ORC_E_LEN;
  uint64_t off = 4;
  double error = r_f64(src + off);
  off += 8;
  double adjustment = r_f64(src + off);
  off += 8;
  double height = r_f64(src + off);
  off += 8;
  for (uint64_t i = 0; i < num_portion; ++i, off += 8) row[i] = r_f64(src + off);
  row[num_portion] = error;
  row[num_portion + 1] = adjustment;
  row[num_portion + 2] = height;
  *dim = (uint32_t)num_portion;
  return 0;
}

/* SmolStr / Bytes (transformable 0.1): u32 BE byte length | bytes */
static uint32_t put_bytes(uint8_t* d, const uint8_t* blob, uint64_t off, uint32_t n) {
  w_u32(d, n);
  memcpy(d + 4, blob + off, n);
  return 4 + n;
}
static int get_bytes(const uint8_t* src, uint64_t src_len, uint64_t* o, uint32_t* n) {
  if (src_len < 4) return ORC_E_SHORT;
  uint32_t len = r_u32(src);
  if (src_len - 4 < len) return ORC_E_SHORT;
  *o = 4;
  *n = len;
  return 0;
}

uint32_t orc_wire_frame_len(const orc_wire_msg* m) {
  switch (m->type) {
    case ORC_MSG_JOIN: return 1 + 4 + orc_varint_len(m->ltime) + 4 + m->a_len;        /* join.rs:132-134 */
    case ORC_MSG_LEAVE: return 1 + 4 + 1 + 4 + m->a_len + orc_varint_len(m->ltime);   /* leave.rs:88-90 */
    case ORC_MSG_USER_EVENT:                                                        /* user_event.rs:330-332 */
      return 1 + 4 + orc_varint_len(m->ltime) + 4 + m->a_len + 4 + m->b_len + 1;
    default: return 0;
  }
}

/* raw[0] = tag; encode_message(&msg, &mut raw[1..])  (base.rs:373, api.rs:293) */
uint32_t orc_wire_encode(const orc_wire_msg* m, const uint8_t* blob, uint8_t* dst) {
  uint32_t total = orc_wire_frame_len(m);
  if (!total) return 0;
  dst[0] = m->type;
  uint8_t* b = dst + 1;
  uint32_t off = 0;
  w_u32(b, total - 1); /* encoded_len of the message */
  off += 4;
  if (m->type == ORC_MSG_JOIN) { /* join.rs:82-104 */
    off += orc_varint_encode(m->ltime, b + off);
    off += put_bytes(b + off, blob, m->a_off, m->a_len);
  } else if (m->type == ORC_MSG_LEAVE) { /* leave.rs:62-86 */
    b[off++] = m->flag ? 1 : 0;
    off += orc_varint_encode(m->ltime, b + off);
    off += put_bytes(b + off, blob, m->a_off, m->a_len);
  } else { /* user_event.rs:306-328 */
    b[off++] = m->flag ? 1 : 0;
    off += orc_varint_encode(m->ltime, b + off);
    off += put_bytes(b + off, blob, m->a_off, m->a_len);
    off += put_bytes(b + off, blob, m->b_off, m->b_len);
  }
  return 1 + off;
}

void orc_wire_decode(const uint8_t* buf, uint64_t fo, uint64_t flen, orc_wire_msg* m) {
  memset(m, 0, sizeof(*m));
  if (flen == 0) { /* notify_message: an empty message is ignored (delegate.rs:158-161) */
    m->status = ORC_SKIPPED;
    return;
  }
  const uint8_t* src = buf + fo + 1; /* decode_message(ty, &msg[1..]) */
  uint64_t n = flen - 1, base = fo + 1, o, sl;
  uint32_t len, rd, slen;
  int err = 0;
  m->type = buf[fo];
  switch (m->type) {
    case ORC_MSG_JOIN: /* JoinMessage::decode  join.rs:106-130 */
      if (n < 4) { m->status = ORC_E_SHORT; return; }
      len = r_u32(src);
      if (n < len) { m->status = ORC_E_SHORT; return; }
      o = 4;
      if (!(rd = orc_varint_decode(src + o, n - o, &m->ltime, &err))) { m->status = err; return; }
      o += rd;
      if ((err = get_bytes(src + o, n - o, &sl, &slen))) { m->status = err; return; }
      m->a_off = base + o + sl;
      m->a_len = slen;
      m->frame_len = 1 + len;
      return;
    case ORC_MSG_LEAVE: /* LeaveMessage::decode  leave.rs:92-120 */
      if (n < 5) { m->status = ORC_E_SHORT; return; }
      len = r_u32(src);
      if (n + 5 < len) { m->status = ORC_E_SHORT; return; }
      m->flag = src[4] != 0;
      o = 5;
      if (!(rd = orc_varint_decode(src + o, n - o, &m->ltime, &err))) { m->status = err; return; }
      o += rd;
      if ((err = get_bytes(src + o, n - o, &sl, &slen))) { m->status = err; return; }
      m->a_off = base + o + sl;
      m->a_len = slen;
      m->frame_len = (uint32_t)(1 + o + 4 + slen); /* Ok((offset, ..)) */
      return;
    case ORC_MSG_USER_EVENT: /* UserEventMessage::decode  user_event.rs:334-370 */
      if (n < 4) { m->status = ORC_E_SHORT; return; }
      len = r_u32(src);
      if (n < len) { m->status = ORC_E_SHORT; return; }
      if (n < 5) { m->status = ORC_E_SHORT; return; } /* src[4] would be out of bounds */
      m->flag = src[4] != 0;
      o = 5;
      if (!(rd = orc_varint_decode(src + o, n - o, &m->ltime, &err))) { m->status = err; return; }
      o += rd;
      if ((err = get_bytes(src + o, n - o, &sl, &slen))) { m->status = err; return; }
      m->a_off = base + o + sl;
      m->a_len = slen;
      o += sl + slen;
      if ((err = get_bytes(src + o, n - o, &sl, &slen))) { m->status = err; return; }
      m->b_off = base + o + sl;
      m->b_len = slen;
      m->frame_len = 1 + len;
      return;
    default:
      m->status = ORC_E_TYPE;
      return;
  }
}

/* ------------------------------------------------------------------------ */
/* UserEventCoalescer  core/src/coalesce/user.rs:52-97                      */
/* ------------------------------------------------------------------------ */
uint32_t orc_coalesce_user_events(const orc_uevent* in, uint32_t n, orc_uevent* out) {
  /* IndexMap<name, LatestUserEvents>: names kept in first-insertion order.
   * An event survives to the flush iff its ltime equals its name's final
   * latest ltime (older ones are dropped or cleared, equal ones appended). */
  uint32_t* names = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  uint64_t* lt = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  uint32_t* grp = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  uint32_t nn = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t j = 0;
    while (j < nn && names[j] != in[i].name) ++j;
    grp[i] = j;
    if (j == nn) {
      names[nn] = in[i].name;
      lt[nn++] = in[i].ltime;
    } else if (lt[j] < in[i].ltime) {
      lt[j] = in[i].ltime;
    }
  }
  uint32_t o = 0;
  for (uint32_t j = 0; j < nn; ++j)
    for (uint32_t i = 0; i < n; ++i)
      if (grp[i] == j && in[i].ltime == lt[j]) out[o++] = in[i];
  free(names);
  free(lt);
  free(grp);
  return o;
}

/* ======================================================================
 * memberlist SWIM model.  PARITY UNPINNED: memberlist-core 0.2
 * is not vendored (reference Cargo.toml:27-29; call sites core/src/serf/base.rs:208-225).
 * States: 0 alive, 1 suspect, 2 dead, 3 left, 255 unknown.  Flags: 1 rebroadcast,
 * 2 refute, 4 notify join, 8 notify leave, 16 suspicion started, 32 confirmation.
 * ====================================================================== */
enum { SW_ALIVE = 0, SW_SUSPECT = 1, SW_DEAD = 2, SW_LEFT = 3, SW_UNKNOWN = 255 };

int orc_swim_init(orc_swim* w, uint64_t lo, uint64_t n_loc, uint32_t S, uint32_t k, const uint32_t* timeout,
                  const uint32_t* subject_member, const uint8_t* state0, const uint32_t* inc0, uint32_t self_inc0) {
  memset(w, 0, sizeof(*w));
  w->lo = lo;
  w->n_loc = n_loc;
  w->S = S;
  w->k = k;
  for (int i = 0; i < 5; ++i) w->timeout[i] = timeout[i];
  uint64_t ne = n_loc * S;
  w->state = malloc(ne);
  w->inc = malloc(ne * 4);
  w->change = calloc(ne, 4);
  w->nconf = calloc(ne, 1);
  w->accuser = calloc(ne * 5, 4);
  w->self_inc = malloc(n_loc * 4);
  w->left = calloc(n_loc, 1);
  w->subject_member = malloc((size_t)S * 4);
  if (!w->state || !w->inc || !w->change || !w->nconf || !w->accuser || !w->self_inc || !w->left ||
      !w->subject_member)
    return -1;
  memcpy(w->subject_member, subject_member, (size_t)S * 4);
  for (uint64_t r = 0; r < n_loc; ++r) {
    w->self_inc[r] = self_inc0;
    for (uint32_t s = 0; s < S; ++s) {
      w->state[r * S + s] = state0[s];
      w->inc[r * S + s] = inc0[s];
    }
  }
  return 0;
}

void orc_swim_free(orc_swim* w) {
  free(w->state);
  free(w->inc);
  free(w->change);
  free(w->nconf);
  free(w->accuser);
  free(w->self_inc);
  free(w->left);
  free(w->subject_member);
  memset(w, 0, sizeof(*w));
}

void orc_swim_set_left(orc_swim* w, uint64_t member, uint8_t left) { w->left[member - w->lo] = left; }

/* refute(me, accusedInc): inc = nextIncarnation(); if accusedInc >= inc,
 * inc = skipIncarnation(accusedInc - inc + 1); me.Incarnation = inc */
static uint32_t sw_refute_o(orc_swim* w, uint64_t r, uint64_t e, uint32_t accused) {
  uint32_t inc = ++w->self_inc[r];
  if (accused >= inc) {
    w->self_inc[r] += accused - inc + 1;
    inc = w->self_inc[r];
  }
  w->inc[e] = inc;
  return inc;
}

/* aliveNode(a, notify, bootstrap=false).  A node never heard of is first added to
 * nodeMap as StateDead with incarnation 0, then the incarnation checks run. */
static int sw_alive_node(orc_swim* w, uint64_t r, uint64_t e, int is_local, uint32_t a_inc, uint32_t now,
                         uint32_t* ref) {
  if (w->state[e] == SW_UNKNOWN) {
    w->state[e] = SW_DEAD;
    w->inc[e] = 0;
    w->change[e] = 0;
    w->nconf[e] = 0;
  }
  if (a_inc <= w->inc[e] && !is_local) return 0;  /* old incarnation, not about us */
  if (a_inc < w->inc[e] && is_local) return 0;    /* strictly older, about us */
  w->nconf[e] = 0;                                /* delete(m.nodeTimers, a.Node) */
  uint8_t old_state = w->state[e];
  int flags = 0;
  if (is_local) {
    if (a_inc == w->inc[e]) return 0; /* same incarnation and (model) same meta: nothing to refute */
    *ref = sw_refute_o(w, r, e, a_inc);
    flags |= 2;
  } else {
    flags |= 1;
    w->inc[e] = a_inc;
    if (w->state[e] != SW_ALIVE) {
      w->state[e] = SW_ALIVE;
      w->change[e] = now;
    }
  }
  if (old_state == SW_DEAD || old_state == SW_LEFT) flags |= 4; /* NotifyJoin */
  return flags;
}

/* suspectNode(s) */
static int sw_suspect_node(orc_swim* w, uint64_t r, uint64_t e, int is_local, uint32_t s_inc, uint32_t from,
                           uint32_t now, uint32_t* ref) {
  if (w->state[e] == SW_UNKNOWN) return 0;
  if (s_inc < w->inc[e]) return 0;
  if (w->state[e] == SW_SUSPECT) { /* timer exists: timer.Confirm(s.From) */
    uint32_t n = w->nconf[e];
    if (n >= w->k) return 0;
    uint32_t* acc = w->accuser + e * 5;
    for (uint32_t i = 0; i <= n; ++i)
      if (acc[i] == from) return 0;
    acc[n + 1] = from;
    w->nconf[e] = (uint8_t)(n + 1);
    return 1 | 32;
  }
  if (w->state[e] != SW_ALIVE) return 0;
  if (is_local) {
    *ref = sw_refute_o(w, r, e, s_inc);
    return 2;
  }
  w->inc[e] = s_inc;
  w->state[e] = SW_SUSPECT;
  w->change[e] = now;
  w->accuser[e * 5] = from;
  w->nconf[e] = 0;
  return 1 | 16;
}

/* deadNode(d) */
static int sw_dead_node(orc_swim* w, uint64_t r, uint64_t e, int is_local, uint32_t d_inc, int node_is_from,
                        uint32_t now, uint32_t* ref) {
  if (w->state[e] == SW_UNKNOWN) return 0;
  if (d_inc < w->inc[e]) return 0;
  w->nconf[e] = 0; /* delete(m.nodeTimers, d.Node) */
  if (w->state[e] == SW_DEAD || w->state[e] == SW_LEFT) return 0;
  if (is_local && !w->left[r]) {
    *ref = sw_refute_o(w, r, e, d_inc);
    return 2;
  }
  w->inc[e] = d_inc;
  w->state[e] = node_is_from ? SW_LEFT : SW_DEAD;
  w->change[e] = now;
  return 1 | 8;
}

void orc_swim_apply(orc_swim* w, const orc_swim_msg* m, uint64_t n, uint32_t now, int32_t* flags, uint32_t* refute_inc) {
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t r = m[i].receiver - w->lo, e = r * w->S + m[i].subject;
    uint32_t node = w->subject_member[m[i].subject];
    int is_local = node == m[i].receiver;
    uint32_t ref = 0;
    int f = 0;
    switch (m[i].type) {
      case 0: f = sw_alive_node(w, r, e, is_local, m[i].incarnation, now, &ref); break;
      case 1: f = sw_suspect_node(w, r, e, is_local, m[i].incarnation, m[i].from, now, &ref); break;
      case 2: f = sw_dead_node(w, r, e, is_local, m[i].incarnation, node == m[i].from, now, &ref); break;
      default: break;
    }
    flags[i] = f;
    if (refute_inc) refute_inc[i] = ref;
  }
}

/* suspicion timeout: the timer fires once now - start >= timeout(confirmations) and runs
 * deadNode{Incarnation: state.Incarnation, Node, From: m.config.Name} */
uint64_t orc_swim_tick(orc_swim* w, uint32_t now) {
  uint64_t fired = 0;
  for (uint64_t r = 0; r < w->n_loc; ++r)
    for (uint32_t s = 0; s < w->S; ++s) {
      uint64_t e = r * w->S + s;
      if (w->state[e] != SW_SUSPECT) continue;
      uint32_t c = w->nconf[e] <= w->k ? w->nconf[e] : w->k;
      if (now - w->change[e] < w->timeout[c]) continue;
      uint32_t me = (uint32_t)(w->lo + r), node = w->subject_member[s], ref = 0;
      sw_dead_node(w, r, e, node == me, w->inc[e], node == me, now, &ref);
      fired++;
    }
  return fired;
}

void orc_swim_dump(const orc_swim* w, uint64_t first, uint64_t count, uint8_t* state, uint32_t* inc, uint32_t* change,
                   uint8_t* nconf, uint32_t* self_inc) {
  for (uint64_t i = 0; i < count * w->S; ++i) {
    uint64_t e = first * w->S + i;
    int known = w->state[e] != SW_UNKNOWN;
    state[i] = w->state[e];
    inc[i] = known ? w->inc[e] : 0;
    change[i] = known ? w->change[e] : 0;
    nconf[i] = w->state[e] == SW_SUSPECT ? w->nconf[e] : 0;
  }
  for (uint64_t r = 0; r < count; ++r) self_inc[r] = w->self_inc[first + r];
}

/* ------------------------------------------------------------------------ */
/* Snapshot log (core/src/snapshot.rs) and Reconnector (base.rs:632-701)    */
/* ------------------------------------------------------------------------ */
#define PURPOSE_RECONNECT 7u
#define SNAP_BYTES_PER_NODE 128u   /* snapshot.rs:56 */
#define SNAP_COMPACTION_THRESHOLD 2u /* snapshot.rs:60 */

static void le64(uint8_t* d, uint64_t v) {
  for (int i = 0; i < 8; ++i, v >>= 8) d[i] = (uint8_t)v;
}
static uint64_t rd_le64(const uint8_t* s) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | s[i];
  return v;
}
static uint32_t rd_le32(const uint8_t* s) { return (uint32_t)s[0] | (uint32_t)s[1] << 8 | (uint32_t)s[2] << 16 | (uint32_t)s[3] << 24; }

/* SnapshotRecord::encode (snapshot.rs:159-218): node records [tag][u32 LE len][node],
 * clock records [tag][u64 LE], others [tag].  Returns the bytes written (out may be NULL). */
static uint32_t snap_rec_node(uint8_t* out, uint8_t tag, uint32_t subj) {
  if (out) {
    out[0] = tag;
    out[1] = 4;
    out[2] = out[3] = out[4] = 0;
    out[5] = (uint8_t)subj;
    out[6] = (uint8_t)(subj >> 8);
    out[7] = (uint8_t)(subj >> 16);
    out[8] = (uint8_t)(subj >> 24);
  }
  return 9;
}
static uint32_t snap_rec_clock(uint8_t* out, uint8_t tag, uint64_t t) {
  if (out) {
    out[0] = tag;
    le64(out + 1, t);
  }
  return 9;
}

int orc_snapshot_replay(const uint8_t* f, uint64_t len, int rejoin, uint32_t s, uint32_t* alive, uint64_t clocks[3]) {
  const uint32_t words = (s + 31) / 32;
  memset(alive, 0, (size_t)words * 4);
  clocks[0] = clocks[1] = clocks[2] = 0;
  uint64_t p = 0;
  while (p < len) {
    const uint8_t tag = f[p++];
    switch (tag) {
      case ORC_SNAP_ALIVE:
      case ORC_SNAP_NOT_ALIVE: {
        if (len - p < 4) return ORC_SNAP_ERR_TRUNCATED;
        uint32_t n = rd_le32(f + p);
        p += 4;
        if (len - p < n) return ORC_SNAP_ERR_TRUNCATED;
        if (n != 4) return ORC_SNAP_ERR_NODE; /* TransformDelegate::decode_node fails */
        uint32_t subj = rd_le32(f + p);
        p += 4;
        if (subj >= s) return ORC_SNAP_ERR_NODE;
        if (tag == ORC_SNAP_ALIVE) alive[subj >> 5] |= 1u << (subj & 31);
        else alive[subj >> 5] &= ~(1u << (subj & 31));
        break;
      }
      case ORC_SNAP_CLOCK:
      case ORC_SNAP_EVENT_CLOCK:
      case ORC_SNAP_QUERY_CLOCK:
        if (len - p < 8) return ORC_SNAP_ERR_TRUNCATED;
        clocks[tag - ORC_SNAP_CLOCK] = rd_le64(f + p);
        p += 8;
        break;
      case ORC_SNAP_COORDINATE:
      case ORC_SNAP_COMMENT: break;
      case ORC_SNAP_LEAVE: /* ignored when re-joining after a leave (snapshot.rs:324-334) */
        if (rejoin) break;
        memset(alive, 0, (size_t)words * 4);
        clocks[0] = clocks[1] = clocks[2] = 0;
        break;
      default: return ORC_SNAP_ERR_RECORD; /* UnknownRecordType */
    }
  }
  return 0;
}

/* ---- the in-memory Snapshotter */
static int snap_put(orc_snapshotter* sp, const uint8_t* rec, uint32_t n) {
  if (sp->len + n > sp->cap) {
    uint64_t c = sp->cap ? sp->cap * 2 : 256;
    while (c < sp->len + n) c *= 2;
    uint8_t* b = (uint8_t*)realloc(sp->buf, c);
    if (!b) return -1;
    sp->buf = b;
    sp->cap = c;
  }
  memcpy(sp->buf + sp->len, rec, n);
  sp->len += n;
  return 0;
}

static uint64_t snap_popcount(const orc_snapshotter* sp) {
  uint64_t c = 0;
  for (uint32_t i = 0; i < (sp->s + 31) / 32; ++i) c += (uint64_t)__builtin_popcount(sp->alive[i]);
  return c;
}

/* compact (snapshot.rs:786-880): the alive nodes, then the three clocks */
static void snap_compact(orc_snapshotter* sp) {
  uint8_t rec[9];
  sp->len = 0;
  for (uint32_t subj = 0; subj < sp->s; ++subj)
    if (sp->alive[subj >> 5] >> (subj & 31) & 1) snap_put(sp, rec, snap_rec_node(rec, ORC_SNAP_ALIVE, subj));
  snap_put(sp, rec, snap_rec_clock(rec, ORC_SNAP_CLOCK, sp->last_clock));
  snap_put(sp, rec, snap_rec_clock(rec, ORC_SNAP_EVENT_CLOCK, sp->last_event_clock));
  snap_put(sp, rec, snap_rec_clock(rec, ORC_SNAP_QUERY_CLOCK, sp->last_query_clock));
  sp->offset = sp->len;
  sp->compactions++;
}

/* try_append / append_line (snapshot.rs:722-776): write, then compact past
 * max(alive * 128 * 2, min_compact_size) (snapshot_max_size, 778-784) */
static void snap_append(orc_snapshotter* sp, const uint8_t* rec, uint32_t n) {
  if (snap_put(sp, rec, n)) return;
  sp->offset += n;
  uint64_t th = snap_popcount(sp) * SNAP_BYTES_PER_NODE * SNAP_COMPACTION_THRESHOLD;
  if (th < sp->min_compact) th = sp->min_compact;
  if (sp->offset > th) snap_compact(sp);
}

int orc_snapshotter_open(orc_snapshotter* sp, uint32_t s, const uint8_t* file, uint64_t len, uint64_t min_compact,
                         int rejoin) {
  memset(sp, 0, sizeof(*sp));
  sp->s = s;
  sp->alive = (uint32_t*)calloc((s + 31) / 32 + 1, 4);
  if (!sp->alive) return -1;
  uint64_t clocks[3] = {0, 0, 0};
  if (len) {
    int rc = orc_snapshot_replay(file, len, rejoin, s, sp->alive, clocks);
    if (rc) return rc;
    if (snap_put(sp, file, (uint32_t)len)) return -1;
  }
  sp->offset = len;
  sp->last_clock = clocks[0];
  sp->last_event_clock = clocks[1];
  sp->last_query_clock = clocks[2];
  sp->min_compact = min_compact;
  sp->rejoin = rejoin;
  return 0;
}

void orc_snapshotter_free(orc_snapshotter* sp) {
  free(sp->buf);
  free(sp->alive);
  memset(sp, 0, sizeof(*sp));
}

void orc_snapshotter_user_event(orc_snapshotter* sp, uint64_t ltime) {
  if (sp->leaving || ltime <= sp->last_event_clock) return; /* stream_flush_event!: stop after a leave */
  sp->last_event_clock = ltime;
  uint8_t rec[9];
  snap_append(sp, rec, snap_rec_clock(rec, ORC_SNAP_EVENT_CLOCK, ltime));
}

void orc_snapshotter_query(orc_snapshotter* sp, uint64_t ltime) {
  if (sp->leaving || ltime <= sp->last_query_clock) return;
  sp->last_query_clock = ltime;
  uint8_t rec[9];
  snap_append(sp, rec, snap_rec_clock(rec, ORC_SNAP_QUERY_CLOCK, ltime));
}

/* update_clock (snapshot.rs:713-720): last_seen = clock.time() - 1 (saturating) */
void orc_snapshotter_update_clock(orc_snapshotter* sp, uint64_t clock_time) {
  uint64_t last_seen = clock_time ? clock_time - 1 : 0;
  if (last_seen > sp->last_clock) {
    sp->last_clock = last_seen;
    uint8_t rec[9];
    snap_append(sp, rec, snap_rec_clock(rec, ORC_SNAP_CLOCK, last_seen));
  }
}

void orc_snapshotter_member_event(orc_snapshotter* sp, uint32_t ev, uint32_t subj, uint64_t clock_time) {
  if (sp->leaving || subj >= sp->s) return;
  uint8_t rec[9];
  if (ev == EV_JOIN) {
    sp->alive[subj >> 5] |= 1u << (subj & 31);
    snap_append(sp, rec, snap_rec_node(rec, ORC_SNAP_ALIVE, subj));
  } else if (ev == EV_LEAVE || ev == EV_FAILED) {
    sp->alive[subj >> 5] &= ~(1u << (subj & 31));
    snap_append(sp, rec, snap_rec_node(rec, ORC_SNAP_NOT_ALIVE, subj));
  }
  orc_snapshotter_update_clock(sp, clock_time);
}

/* handle_leave (snapshot.rs:568-586) */
void orc_snapshotter_leave(orc_snapshotter* sp) {
  sp->leaving = 1;
  if (!sp->rejoin) memset(sp->alive, 0, (size_t)((sp->s + 31) / 32) * 4);
  uint8_t rec = ORC_SNAP_LEAVE;
  snap_append(sp, &rec, 1);
}

/* ---- the world's snapshotters */
int orc_world_enable_snapshot(orc_world* w, int rejoin_after_leave) {
  free(w->snap_bits);
  free(w->snap_sn);
  w->snap_w = (w->s + 31) / 32;
  w->snap_bits = (uint32_t*)calloc((size_t)w->n * w->snap_w, 4);
  w->snap_sn = (uint64_t*)calloc((size_t)w->n * 4, 8);
  if (!w->snap_bits || !w->snap_sn) return -1;
  w->snap_rejoin = rejoin_after_leave;
  for (uint32_t m = 0; m < w->n; ++m)
    for (uint32_t subj = 0; subj < w->s; ++subj) {
      size_t e = (size_t)m * w->s + subj;
      if (w->v_kind[e] == ORC_K_KNOWN && (w->v_status[e] == ORC_ST_ALIVE || w->v_status[e] == ORC_ST_LEAVING))
        w->snap_bits[(size_t)m * w->snap_w + (subj >> 5)] |= 1u << (subj & 31);
    }
  return 0;
}

/* Snapshot::leave at Serf::leave: the clock ticker's last value, then recording stops */
static void snap_leave(orc_world* w, uint32_t m) {
  uint64_t* sn = w->snap_sn + (size_t)m * 4;
  if (sn[3] & 1) return;
  sn[2] = w->clock[m] ? w->clock[m] - 1 : 0;
  sn[3] |= 1;
  if (!w->snap_rejoin) memset(w->snap_bits + (size_t)m * w->snap_w, 0, (size_t)w->snap_w * 4);
}

uint64_t orc_world_snapshot_encode(const orc_world* w, uint32_t m, uint8_t* out) {
  if (!w->snap_bits) return 0;
  const uint32_t* bits = w->snap_bits + (size_t)m * w->snap_w;
  const uint64_t* sn = w->snap_sn + (size_t)m * 4;
  const uint64_t now_clock = w->clock[m] ? w->clock[m] - 1 : 0;
  const int leaving = (int)(sn[3] & 1);
  uint64_t p = 0;
  for (uint32_t subj = 0; subj < w->s; ++subj)
    if (bits[subj >> 5] >> (subj & 31) & 1) p += snap_rec_node(out ? out + p : NULL, ORC_SNAP_ALIVE, subj);
  p += snap_rec_clock(out ? out + p : NULL, ORC_SNAP_CLOCK, leaving ? sn[2] : now_clock);
  p += snap_rec_clock(out ? out + p : NULL, ORC_SNAP_EVENT_CLOCK, sn[0]);
  p += snap_rec_clock(out ? out + p : NULL, ORC_SNAP_QUERY_CLOCK, sn[1]);
  if (leaving) {
    if (out) out[p] = ORC_SNAP_LEAVE;
    p += 1;
    /* the shutdown's update_clock (snapshot.rs:622-623) */
    if (now_clock > sn[2]) p += snap_rec_clock(out ? out + p : NULL, ORC_SNAP_CLOCK, now_clock);
  }
  return p;
}

int orc_world_restart(orc_world* w, uint32_t m, const uint8_t* file, uint64_t len) {
  if (!w->snap_bits || m >= w->n) return -1;
  uint32_t* bits = w->snap_bits + (size_t)m * w->snap_w;
  uint64_t old[3];
  uint32_t* tmp = (uint32_t*)calloc(w->snap_w + 1, 4);
  if (!tmp) return -1;
  int rc = orc_snapshot_replay(file, len, w->snap_rejoin, w->s, tmp, old);
  if (!rc) memcpy(bits, tmp, (size_t)w->snap_w * 4); /* a file that does not replay changes nothing */
  free(tmp);
  if (rc) return rc;
  /* Serf::new (base.rs:122-204): clocks start at 1, then witness the replayed ones;
   * events / queries older than the snapshot are ignored from now on */
  w->clock[m] = w->eclock[m] = w->qclock[m] = 1;
  orc_clock_witness(&w->clock[m], old[0]);
  orc_clock_witness(&w->eclock[m], old[1]);
  orc_clock_witness(&w->qclock[m], old[2]);
  w->emin[m] = old[1] + 1;
  w->qmin[m] = old[2] + 1;
  w->serf_state[m] = ORC_SERF_ALIVE;
  /* a fresh process: no member states, intents, queued broadcasts, event / query buffers */
  for (uint32_t subj = 0; subj < w->s; ++subj) erase_entry(w, (size_t)m * w->s + subj);
  for (uint32_t i = 0; i < 3 * w->qcap; ++i) {
    size_t q = (size_t)m * 3 * w->qcap + i;
    w->q_rumor[q] = EMPTY_RUMOR;
    w->q_seq[q] = 0;
    w->q_tx[q] = 0;
    w->q_len[q] = 0;
  }
  for (uint32_t q = 0; q < 3; ++q) w->q_next_seq[(size_t)m * 3 + q] = w->q_hwm[(size_t)m * 3 + q] = w->q_hole[(size_t)m * 3 + q] = 0;
  memset(w->eb_ltime + (size_t)m * w->ebuf, 0, (size_t)w->ebuf * 8);
  memset(w->eb_cnt + (size_t)m * w->ebuf, 0, (size_t)w->ebuf * 4);
  memset(w->eb_keys + (size_t)m * w->ebuf * w->slot_k, 0, (size_t)w->ebuf * w->slot_k * 8);
  memset(w->qb_ltime + (size_t)m * w->qbuf, 0, (size_t)w->qbuf * 8);
  memset(w->qb_cnt + (size_t)m * w->qbuf, 0, (size_t)w->qbuf * 4);
  memset(w->qb_ids + (size_t)m * w->qbuf * w->slot_k, 0, (size_t)w->qbuf * w->slot_k * 4);
  if (w->member_subj[m] >= 0) w->refute_cnt[w->member_subj[m]] = 0;
  uint64_t* sn = w->snap_sn + (size_t)m * 4;
  sn[0] = old[1];
  sn[1] = old[2];
  sn[2] = 0;
  sn[3] = 0;
  /* handle_rejoin (base.rs:1741-1770): memberlist.join to the replayed nodes until one
   * answers; memberlist's state exchange then notifies a join of every live member */
  int joined = 0;
  for (uint32_t subj = 0; subj < w->s && !joined; ++subj)
    if ((bits[subj >> 5] >> (subj & 31) & 1) && (int32_t)subj != w->member_subj[m] && w->alive[w->subj_member[subj]])
      joined = 1;
  if (joined)
    for (uint32_t subj = 0; subj < w->s; ++subj)
      if ((int32_t)subj != w->member_subj[m] && w->alive[w->subj_member[subj]]) orc_handle_node_join(w, m, subj);
  return joined;
}

/* Reconnector throttle (base.rs:670-671):
 * num_alive = (states.len() - num_failed - left_members.len()).max(1);
 * prob = num_failed as f32 / num_alive as f32 (usize -> f32 rounds to nearest) */
float orc_reconnect_prob(uint64_t states, uint64_t failed, uint64_t left) {
  uint64_t alive = states - failed - left;
  if (alive < 1) alive = 1;
  return (float)failed / (float)alive;
}

uint32_t orc_world_reconnect(orc_world* w, uint32_t tick, uint32_t* target) {
  uint32_t key[2];
  seed_key(w->seed, key);
  uint32_t joins = 0;
  for (uint32_t m = 0; m < w->n; ++m) {
    target[m] = EMPTY_RUMOR;
    if (!w->alive[m]) continue;
    const size_t row = (size_t)m * w->s;
    /* members.states.len(): the n - s untracked members (implicitly Alive; the local node
     * is one of them unless it is a subject), the local node if it is a subject, and the
     * tracked subjects it knows */
    const uint64_t known = orc_states_len(w, m);
    uint32_t failed = 0, left = 0;
    for (uint32_t subj = 0; subj < w->s; ++subj) {
      if ((int32_t)subj == w->member_subj[m] || w->v_kind[row + subj] != ORC_K_KNOWN) continue;
      failed += w->v_status[row + subj] == ORC_ST_FAILED;
      left += w->v_status[row + subj] == ORC_ST_LEFT;
    }
    if (!failed) continue;
    const float prob = orc_reconnect_prob(known, failed, left);
    uint32_t ctr[4] = {0, PURPOSE_RECONNECT << 24, m, tick}, o[4];
    orc_philox4x32(ctr, key, o);
    const float r = (float)(o[0] >> 8) * (1.0f / 16777216.0f); /* rng.gen::<f32>() */
    if (r > prob) continue;
    uint32_t idx = (uint32_t)(((uint64_t)o[1] * failed) >> 32); /* gen_range(0..num_failed) */
    for (uint32_t subj = 0; subj < w->s; ++subj) {
      if ((int32_t)subj == w->member_subj[m] || w->v_kind[row + subj] != ORC_K_KNOWN ||
          w->v_status[row + subj] != ORC_ST_FAILED)
        continue;
      if (idx-- == 0) {
        target[m] = subj;
        break;
      }
    }
    if (w->alive[w->subj_member[target[m]]]) {
      orc_handle_node_join(w, m, target[m]);
      joins++;
    }
  }
  return joins;
}

/* ---- MemberEventCoalescer  coalesce/member.rs:60-118 -------------------------------- */
typedef struct {
  uint64_t key; /* group << 32 | node */
  uint64_t arrival;
} mc_item;
static int mc_cmp(const void* a, const void* b) {
  const mc_item *x = (const mc_item*)a, *y = (const mc_item*)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return x->arrival < y->arrival ? -1 : (x->arrival > y->arrival);
}
static int mc_out_cmp(const void* a, const void* b) {
  const orc_mevent *x = (const orc_mevent*)a, *y = (const orc_mevent*)b;
  if (x->group != y->group) return x->group < y->group ? -1 : 1;
  if (x->type != y->type) return x->type < y->type ? -1 : 1;
  return x->node < y->node ? -1 : (x->node > y->node);
}
uint64_t orc_member_coalesce(uint8_t* last, uint32_t n_nodes, const orc_mevent* in, uint64_t n, orc_mevent* out) {
  if (!n) return 0;
  mc_item* it = (mc_item*)malloc(n * sizeof(mc_item));
  if (!it) return 0;
  for (uint64_t i = 0; i < n; ++i) {
    it[i].key = ((uint64_t)in[i].group << 32) | in[i].node;
    it[i].arrival = i;
  }
  qsort(it, n, sizeof(mc_item), mc_cmp);
  uint64_t k = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (i + 1 < n && it[i + 1].key == it[i].key) continue; /* latest_events.insert: the last one stays */
    const orc_mevent* e = &in[it[i].arrival];
    uint8_t* lp = last + (size_t)e->group * n_nodes + e->node;
    /* Some(&previous) if previous == cev.ty && cev.ty != Update => continue */
    if (*lp == e->type && e->type != 4u) continue;
    *lp = (uint8_t)e->type; /* self.last_events.insert(id, cev.ty) */
    out[k++] = *e; /* the latest CoalesceEvent's member */
  }
  free(it);
  qsort(out, k, sizeof(orc_mevent), mc_out_cmp);
  return k;
}

/* ---- C1 accuracy: median relative error of estimate_rtt over all pairs ------------ */
static int dbl_cmp(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : (x > y);
}
double orc_vivaldi_pop_median_rel_error(const orc_vivaldi_pop* p) {
  const uint32_t n = p->n, dim = p->opts.dimensionality, st = p->row_stride;
  if (n < 2) return 0.0;
  double *x = (double*)malloc(n * sizeof(double)), *y = (double*)malloc(n * sizeof(double)),
         *h = (double*)malloc(n * sizeof(double));
  const uint64_t pairs = (uint64_t)n * (n - 1) / 2;
  double* rel = (double*)malloc(pairs * sizeof(double));
  if (!x || !y || !h || !rel) {
    free(x), free(y), free(h), free(rel);
    return -1.0;
  }
  for (uint32_t i = 0; i < n; ++i) orc_true_position(p->seed, i, &x[i], &y[i], &h[i]);
  uint64_t k = 0;
  for (uint32_t i = 0; i < n; ++i) {
    orc_coord a;
    row_to_coord(p->rows_cur + (size_t)i * st, dim, &a);
    for (uint32_t j = i + 1; j < n; ++j) {
      orc_coord b;
      row_to_coord(p->rows_cur + (size_t)j * st, dim, &b);
      const double dx = x[i] - x[j], dy = y[i] - y[j];
      const double tr = (double)sat_u64((sqrt(dx * dx + dy * dy) + h[i] + h[j]) * 1.0e9);
      const double est = (double)orc_coord_distance_ns(&a, &b);
      rel[k++] = fabs(est - tr) / tr;
    }
  }
  qsort(rel, k, sizeof(double), dbl_cmp);
  const double med = (k & 1) ? rel[k / 2] : 0.5 * (rel[k / 2 - 1] + rel[k / 2]);
  free(x), free(y), free(h), free(rel);
  return med;
}
