/*
 * knn_ref.c — CPU restatement of fenix's brute-force search, used ONLY as a
 * checker (tests/, __graft_entry__.smoke) and as the timed CPU baseline
 * (bench.py cpu_baseline leg).  TEST INFRASTRUCTURE: the product path
 * (fenix_amd/) never loads this library.
 *
 * What it restates (nrlugg/fenix, paths relative to /root/reference):
 *   src/fenix/io/coder/coder.py:38-50   metric formulas:
 *       l2/euclidean  sqrt(sum (x-q)^2)          (torch.cdist, coder.py:39-40)
 *       cosine        0.5 - 0.5 * (x/max(|x|,1e-12)) . (q/max(|q|,1e-12))
 *                                                (F.normalize + matmul, coder.py:42-45)
 *       dot/inner_product  -(x . q)              (coder.py:47-48)
 *   src/fenix/io/index/index.py:165-168  top-k = select_k_unstable ascending
 *       on __DISTANCE__ (NaN after numbers), here with the deterministic
 *       (distance, row) tie-break of include/fenix_knn.h.
 *   src/fenix/io/index/index.py:161      filter -> a row bitmap (NULL = all).
 * Arithmetic: precision=64 evaluates the formulas in double from the stored
 * f32/f16 values (the "DuckDB-semantics" direct-difference restatement, the
 * parity oracle for row ids); precision=32 evaluates them in float with the
 * same direct formulas (the CPU baseline: DuckDB's array_distance computes
 * in float).
 *
 * The generator fx_ref_fill is the host half of the portable corpus generator
 * (device half: fenix_amd/csrc/knn_util.hip); both are bit-identical.
 * The clustered variant restates the reference test corpus,
 * tests/test_flight.py:21-22 (x = x + 10 * x[0, :] per batch).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static float irwin_hall4(uint64_t h) {
  int s = (int)(h & 0xffff) + (int)((h >> 16) & 0xffff) + (int)((h >> 32) & 0xffff) +
          (int)(h >> 48) - 131070;
  volatile float f = (float)s; /* keep the single rounding of the product */
  return f * 2.6428998e-05f;
}

void fx_ref_fill(float* x, int64_t n, int64_t d, uint64_t seed, int64_t row_base,
                 int64_t cluster) {
  const uint64_t smix = seed * 0x9E3779B97F4A7C15ull;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < n; ++r) {
    const uint64_t g = (uint64_t)(row_base + r);
    const uint64_t b0 = cluster > 0 ? g / (uint64_t)cluster * (uint64_t)cluster : g;
    for (int64_t c = 0; c < d; ++c) {
      float v = irwin_hall4(splitmix64(smix + g * (uint64_t)d + (uint64_t)c));
      if (cluster > 0) {
        volatile float t = 10.0f * irwin_hall4(splitmix64(smix + b0 * (uint64_t)d + (uint64_t)c));
        v = v + t;
      }
      x[r * d + c] = v;
    }
  }
}

static float half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000) << 16;
  uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ff, u;
  if (exp == 0) {
    if (man == 0) {
      u = sign;
    } else { /* subnormal */
      int e = -1;
      do {
        ++e;
        man <<= 1;
      } while ((man & 0x400) == 0);
      u = sign | ((uint32_t)(127 - 15 - e) << 23) | ((man & 0x3ff) << 13);
    }
  } else if (exp == 31) {
    u = sign | 0x7f800000u | (man << 13);
  } else {
    u = sign | ((exp + 127 - 15) << 23) | (man << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}

typedef struct {
  double d;
  int64_t r;
} cand_t;

/* strict (distance, row) order; NaN after every number; -0 == +0 */
static int cand_less(const cand_t* a, const cand_t* b) {
  int an = isnan(a->d), bn = isnan(b->d);
  if (an || bn) {
    if (an && bn) return a->r < b->r;
    return bn;
  }
  if (a->d != b->d) return a->d < b->d;
  return a->r < b->r;
}

/* bounded max-heap of the k best candidates */
static void heap_push(cand_t* h, int64_t* size, int64_t k, cand_t c) {
  if (*size < k) {
    int64_t i = (*size)++;
    h[i] = c;
    while (i > 0) {
      int64_t p = (i - 1) / 2;
      if (cand_less(&h[p], &h[i])) {
        cand_t t = h[p];
        h[p] = h[i];
        h[i] = t;
        i = p;
      } else {
        break;
      }
    }
    return;
  }
  if (!cand_less(&c, &h[0])) return;
  h[0] = c;
  int64_t i = 0;
  for (;;) {
    int64_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < k && cand_less(&h[m], &h[l])) m = l;
    if (r < k && cand_less(&h[m], &h[r])) m = r;
    if (m == i) break;
    cand_t t = h[m];
    h[m] = h[i];
    h[i] = t;
    i = m;
  }
}

static int cmp_cand(const void* a, const void* b) {
  const cand_t* x = (const cand_t*)a;
  const cand_t* y = (const cand_t*)b;
  if (cand_less(x, y)) return -1;
  if (cand_less(y, x)) return 1;
  return 0;
}

static double row_dist64(const float* x, const uint16_t* xh, const float* q, int64_t d, int metric,
                         double qn) {
  double s1 = 0.0, s2 = 0.0;
  for (int64_t c = 0; c < d; ++c) {
    double v = x ? (double)x[c] : (double)half_to_float(xh[c]);
    double w = (double)q[c];
    if (metric == 0) {
      double t = v - w;
      s1 += t * t;
    } else {
      s1 += v * w;
      if (metric == 2) s2 += v * v;
    }
  }
  if (metric == 0) return sqrt(s1);
  if (metric == 1) return -s1;
  double nx = sqrt(s2);
  if (nx < 1e-12) nx = 1e-12;
  return 0.5 - 0.5 * (s1 / (nx * qn));
}

/* f32 direct formulas with 8 independent accumulators (vectorisable without
 * reassociation flags): the CPU baseline arithmetic. */
static double row_dist32(const float* x, const uint16_t* xh, const float* q, int64_t d, int metric,
                         float qn) {
  float a[8] = {0}, b[8] = {0};
  int64_t c = 0;
  if (x) {
    for (; c + 8 <= d; c += 8) {
      for (int j = 0; j < 8; ++j) {
        float v = x[c + j], w = q[c + j];
        if (metric == 0) {
          float t = v - w;
          a[j] += t * t;
        } else {
          a[j] += v * w;
          if (metric == 2) b[j] += v * v;
        }
      }
    }
  }
  float s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < 8; ++j) {
    s1 += a[j];
    s2 += b[j];
  }
  for (; c < d; ++c) {
    float v = x ? x[c] : half_to_float(xh[c]), w = q[c];
    if (metric == 0) {
      float t = v - w;
      s1 += t * t;
    } else {
      s1 += v * w;
      if (metric == 2) s2 += v * v;
    }
  }
  if (metric == 0) return (double)sqrtf(s1);
  if (metric == 1) return (double)(-s1);
  float nx = sqrtf(s2);
  if (nx < 1e-12f) nx = 1e-12f;
  return (double)(0.5f - 0.5f * (s1 / (nx * qn)));
}

/*
 * x: [n][d] (dtype 0 = f32, 1 = f16 bits); q: [nq][d] f32; mask: bitmap or NULL.
 * out_dist/out_row: [nq][k]; slots beyond the admissible rows get NaN / -1.
 * threads <= 0: OpenMP default.  Returns 0, or -1 on bad arguments.
 */
int fx_ref_knn(const void* x, int dtype, int64_t n, int64_t d, int64_t row_base, const float* q,
               int64_t nq, int metric, int64_t k, const uint32_t* mask, int precision,
               int threads, double* out_dist, int64_t* out_row) {
  if (n < 0 || d < 1 || nq < 0 || k < 1 || metric < 0 || metric > 2) return -1;
  if (dtype != 0 && dtype != 1) return -1;
#ifdef _OPENMP
  int nt = threads > 0 ? threads : omp_get_max_threads();
#else
  int nt = 1;
  (void)threads;
#endif
  cand_t* heaps = (cand_t*)malloc(sizeof(cand_t) * (size_t)k * (size_t)nt);
  int64_t* sizes = (int64_t*)calloc((size_t)nt, sizeof(int64_t));
  cand_t* all = (cand_t*)malloc(sizeof(cand_t) * (size_t)k * (size_t)nt);
  if (!heaps || !sizes || !all) {
    free(heaps);
    free(sizes);
    free(all);
    return -1;
  }
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qv = q + qi * d;
    double qn64 = 0.0;
    float qn32 = 0.f;
    for (int64_t c = 0; c < d; ++c) qn64 += (double)qv[c] * (double)qv[c];
    qn64 = sqrt(qn64);
    if (qn64 < 1e-12) qn64 = 1e-12;
    {
      float a[8] = {0};
      int64_t c = 0;
      for (; c + 8 <= d; c += 8)
        for (int j = 0; j < 8; ++j) a[j] += qv[c + j] * qv[c + j];
      for (int j = 0; j < 8; ++j) qn32 += a[j];
      for (; c < d; ++c) qn32 += qv[c] * qv[c];
      qn32 = sqrtf(qn32);
      if (qn32 < 1e-12f) qn32 = 1e-12f;
    }
    memset(sizes, 0, sizeof(int64_t) * (size_t)nt);
#pragma omp parallel num_threads(nt)
    {
#ifdef _OPENMP
      int tid = omp_get_thread_num();
#else
      int tid = 0;
#endif
      cand_t* h = heaps + (size_t)tid * k;
      int64_t hs = 0;
#pragma omp for schedule(static)
      for (int64_t r = 0; r < n; ++r) {
        if (mask && !((mask[r >> 5] >> (r & 31)) & 1u)) continue;
        const float* xf = dtype == 0 ? (const float*)x + r * d : NULL;
        const uint16_t* xh = dtype == 1 ? (const uint16_t*)x + r * d : NULL;
        cand_t c;
        c.d = precision == 32 ? row_dist32(xf, xh, qv, d, metric, qn32)
                              : row_dist64(xf, xh, qv, d, metric, qn64);
        c.r = row_base + r;
        heap_push(h, &hs, k, c);
      }
      sizes[tid] = hs;
    }
    int64_t m = 0;
    for (int t = 0; t < nt; ++t)
      for (int64_t i = 0; i < sizes[t]; ++i) all[m++] = heaps[(size_t)t * k + i];
    qsort(all, (size_t)m, sizeof(cand_t), cmp_cand);
    for (int64_t i = 0; i < k; ++i) {
      if (i < m) {
        out_dist[qi * k + i] = all[i].d;
        out_row[qi * k + i] = all[i].r;
      } else {
        out_dist[qi * k + i] = NAN;
        out_row[qi * k + i] = -1;
      }
    }
  }
  free(heaps);
  free(sizes);
  free(all);
  return 0;
}

/* All distances (the maxval=None / n<=maxval branch of index.py:165). */
int fx_ref_distances(const void* x, int dtype, int64_t n, int64_t d, const float* q, int64_t nq,
                     int metric, int precision, double* out) {
  if (n < 0 || d < 1 || metric < 0 || metric > 2) return -1;
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qv = q + qi * d;
    double qn64 = 0.0;
    for (int64_t c = 0; c < d; ++c) qn64 += (double)qv[c] * (double)qv[c];
    qn64 = sqrt(qn64);
    if (qn64 < 1e-12) qn64 = 1e-12;
    float qn32 = (float)qn64;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n; ++r) {
      const float* xf = dtype == 0 ? (const float*)x + r * d : NULL;
      const uint16_t* xh = dtype == 1 ? (const uint16_t*)x + r * d : NULL;
      out[qi * n + r] = precision == 32 ? row_dist32(xf, xh, qv, d, metric, qn32)
                                        : row_dist64(xf, xh, qv, d, metric, qn64);
    }
  }
  return 0;
}

/* Round-to-nearest-even float -> half bits (the device's __float2half / the
 * fp16 corpus cast, torch .half()); used by fx_ref_knn_gen for fp16 corpora. */
static uint16_t float_to_half(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0u));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520: inf */
  if (a < 0x38800000u) {                                     /* subnormal or zero half */
    if (a < 0x33000000u) return (uint16_t)sign;              /* < 2^-25: rounds to 0 */
    const uint32_t m = (a & 0x7fffffu) | 0x800000u;
    const int sh = 126 - (int)(a >> 23); /* 14..24 */
    uint32_t h = m >> (sh);
    const uint32_t rem = m & ((1u << sh) - 1u), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((a >> 23) - 112u) << 10 | ((a >> 13) & 0x3ffu);
  const uint32_t rem = a & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
  return (uint16_t)(sign | h);
}

/*
 * Top-k over a corpus GENERATED on the fly: row r is fx_ref_fill's row
 * (seed, row_base + r, cluster), rounded to fp16 when as_f16 (the fp16
 * corpora of the tests), except the n_over rows listed in over_rows (local
 * rows, ascending or not), whose values are over_vals[i][d] (f32, or the f32
 * value of an fp16 element).  Corpora of 80M x 768 (configs[3], 246 GB) or
 * 50M x 1536 (configs[4]) are checked this way without holding them in host
 * memory.  Same arithmetic, ordering and outputs as fx_ref_knn.
 */
int fx_ref_knn_gen(uint64_t seed, int64_t row_base, int64_t n, int64_t d, int64_t cluster,
                   int as_f16, const int64_t* over_rows, const float* over_vals, int64_t n_over,
                   const float* q, int64_t nq, int metric, int64_t k, int precision, int threads,
                   double* out_dist, int64_t* out_row) {
  if (n < 0 || d < 1 || nq < 0 || k < 1 || metric < 0 || metric > 2) return -1;
#ifdef _OPENMP
  int nt = threads > 0 ? threads : omp_get_max_threads();
#else
  int nt = 1;
  (void)threads;
#endif
  const int64_t chunk = 1024; /* rows generated per block */
  cand_t* heaps = (cand_t*)malloc(sizeof(cand_t) * (size_t)k * (size_t)nt * (size_t)nq);
  int64_t* sizes = (int64_t*)calloc((size_t)nt * (size_t)nq, sizeof(int64_t));
  cand_t* all = (cand_t*)malloc(sizeof(cand_t) * (size_t)k * (size_t)nt);
  double* qn64 = (double*)malloc(sizeof(double) * (size_t)(nq > 0 ? nq : 1));
  float* qn32 = (float*)malloc(sizeof(float) * (size_t)(nq > 0 ? nq : 1));
  if (!heaps || !sizes || !all || !qn64 || !qn32) {
    free(heaps); free(sizes); free(all); free(qn64); free(qn32);
    return -1;
  }
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qv = q + qi * d;
    double s = 0.0;
    for (int64_t c = 0; c < d; ++c) s += (double)qv[c] * (double)qv[c];
    s = sqrt(s);
    qn64[qi] = s < 1e-12 ? 1e-12 : s;
    float a[8] = {0}, s32 = 0.f;
    int64_t c = 0;
    for (; c + 8 <= d; c += 8)
      for (int j = 0; j < 8; ++j) a[j] += qv[c + j] * qv[c + j];
    for (int j = 0; j < 8; ++j) s32 += a[j];
    for (; c < d; ++c) s32 += qv[c] * qv[c];
    s32 = sqrtf(s32);
    qn32[qi] = s32 < 1e-12f ? 1e-12f : s32;
  }
  const int64_t nblk = (n + chunk - 1) / chunk;
#pragma omp parallel num_threads(nt)
  {
#ifdef _OPENMP
    int tid = omp_get_thread_num();
#else
    int tid = 0;
#endif
    float* rows = (float*)malloc(sizeof(float) * (size_t)chunk * (size_t)d);
#pragma omp for schedule(dynamic, 4)
    for (int64_t b = 0; b < nblk; ++b) {
      const int64_t r0 = b * chunk, m = (n - r0) < chunk ? (n - r0) : chunk;
      fx_ref_fill(rows, m, d, seed, row_base + r0, cluster);
      for (int64_t i = 0; i < n_over; ++i) {
        if (over_rows[i] >= r0 && over_rows[i] < r0 + m)
          memcpy(rows + (over_rows[i] - r0) * d, over_vals + i * d, sizeof(float) * (size_t)d);
      }
      if (as_f16) {
        for (int64_t e = 0; e < m * d; ++e) rows[e] = half_to_float(float_to_half(rows[e]));
      }
      for (int64_t qi = 0; qi < nq; ++qi) {
        cand_t* h = heaps + ((size_t)qi * nt + tid) * k;
        int64_t hs = sizes[(size_t)qi * nt + tid];
        for (int64_t r = 0; r < m; ++r) {
          cand_t c;
          c.d = precision == 32 ? row_dist32(rows + r * d, NULL, q + qi * d, d, metric, qn32[qi])
                                : row_dist64(rows + r * d, NULL, q + qi * d, d, metric, qn64[qi]);
          c.r = row_base + r0 + r;
          heap_push(h, &hs, k, c);
        }
        sizes[(size_t)qi * nt + tid] = hs;
      }
    }
    free(rows);
  }
  for (int64_t qi = 0; qi < nq; ++qi) {
    int64_t m = 0;
    for (int t = 0; t < nt; ++t)
      for (int64_t i = 0; i < sizes[(size_t)qi * nt + t]; ++i)
        all[m++] = heaps[((size_t)qi * nt + t) * k + i];
    qsort(all, (size_t)m, sizeof(cand_t), cmp_cand);
    for (int64_t i = 0; i < k; ++i) {
      out_dist[qi * k + i] = i < m ? all[i].d : NAN;
      out_row[qi * k + i] = i < m ? all[i].r : -1;
    }
  }
  free(heaps); free(sizes); free(all); free(qn64); free(qn32);
  return 0;
}
