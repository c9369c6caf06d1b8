/* Exhaustive checks of two exact fast paths in include/ffd_numerics.h (built and run by
 * tests/test_numerics.py; plain C, -ffp-contract=off):
 *   div  ffd_div_rcp(a, 10, RN(1/10)) == a / 10 for every finite binary32 a >= 0 (the quotient is
 *        odd in a, so this covers the negative half too);
 *   expf ffd_expf_nonpos(x) == ffd_expf(x) bitwise for every binary32 x in [-110, 0] and the edges;
 *   quot ffd_expf_nonpos(ffd_div_rcp_fast(-d, 10, RN(1/10))) == ffd_expf_nonpos(-d / 10) bitwise for every binary32
 *        d in [0, 2^-100] (above it the two quotients are equal: "div").
 * Work is split over threads; prints "ok" or the first mismatch. */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/ffd_numerics.h"

#define NT 8
static volatile int bad = 0;
static uint32_t bad_bits;

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static void* div_worker(void* arg) {
  const uint32_t t = (uint32_t)(uintptr_t)arg, end = 0x7F800000u;
  const float y = 1.0f / 10.0f;
  for (uint32_t u = t; u < end && !bad; u += NT) {
    const float a = f_of(u);
    if (u_of(ffd_div_rcp(a, 10.0f, y)) != u_of(a / 10.0f)) { bad = 1; bad_bits = u; }
  }
  return NULL;
}

static void* exp_worker(void* arg) {
  const uint32_t t = (uint32_t)(uintptr_t)arg, lo = 0x80000000u, hi = u_of(-110.0f);
  for (uint32_t u = lo + t; u <= hi && !bad; u += NT) {
    const float x = f_of(u);
    if (u_of(ffd_expf_nonpos(x)) != u_of(ffd_expf(x))) { bad = 1; bad_bits = u; }
  }
  return NULL;
}

static void* quot_worker(void* arg) {
  const uint32_t t = (uint32_t)(uintptr_t)arg, hi = u_of(0x1p-100f);
  const float y = 1.0f / 10.0f;
  for (uint32_t u = t; u <= hi && !bad; u += NT) {
    const float a = -f_of(u);
    if (u_of(ffd_expf_nonpos(ffd_div_rcp_fast(a, 10.0f, y))) != u_of(ffd_expf_nonpos(a / 10.0f))) { bad = 1; bad_bits = u; }
  }
  return NULL;
}

int main(int argc, char** argv) {
  const int which_div = argc > 1 && strcmp(argv[1], "div") == 0, which_quot = argc > 1 && strcmp(argv[1], "quot") == 0;
  pthread_t th[NT];
  for (uintptr_t t = 0; t < NT; t++)
    pthread_create(&th[t], NULL, which_div ? div_worker : which_quot ? quot_worker : exp_worker, (void*)t);
  for (int t = 0; t < NT; t++) pthread_join(th[t], NULL);
  if (!which_div && !which_quot) {
    const float edge[] = {-INFINITY, -1e30f, -104.0f, nextafterf(-104.0f, -INFINITY), nextafterf(-104.0f, 0.0f), -0.0f};
    for (unsigned i = 0; i < sizeof edge / sizeof edge[0]; i++)
      if (u_of(ffd_expf_nonpos(edge[i])) != u_of(ffd_expf(edge[i]))) { bad = 1; bad_bits = u_of(edge[i]); }
  }
  if (bad) { printf("mismatch at 0x%08x\n", bad_bits); return 1; }
  printf("ok\n");
  return 0;
}
