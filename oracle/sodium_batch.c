/* sodium_batch.c -- TEST / BASELINE INFRASTRUCTURE ONLY (see ntoracle.h).
 *
 * Multi-threaded loop over libsodium's crypto_sign_verify_detached, loaded at
 * run time with dlopen (no link-time dependency: returns -1 when the library is
 * absent).  bench.py's cpu_baseline leg uses it as an external comparator beside
 * the oracle port, without the per-call Python overhead a ctypes loop pays.
 * libsodium 1.0.18's verify coincides with dalek verify_strict on the corpus
 * (SURVEY.md A.4); it is never a parity oracle for verify_batch.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stddef.h>

#include "ntoracle.h"

typedef int (*verify_fn)(const unsigned char *sig, const unsigned char *m, unsigned long long mlen,
                         const unsigned char *pk);

typedef struct {
  verify_fn f;
  const uint8_t *pk, *sig, *msg;
  const uint64_t *off, *len;
  uint64_t lo, hi;
  uint8_t *out;
} sjob;

static void *srun(void *arg) {
  sjob *j = (sjob *)arg;
  for (uint64_t i = j->lo; i < j->hi; ++i)
    j->out[i] = j->f(j->sig + 64 * i, j->msg + j->off[i], j->len[i], j->pk + 32 * i) == 0;
  return NULL;
}

int ntor_sodium_verify_many(const char *libpath, const uint8_t *pk32, const uint8_t *sig64, const uint8_t *msg,
                            const uint64_t *off, const uint64_t *len, uint64_t n, int nthreads, uint8_t *out) {
  void *h = dlopen(libpath, RTLD_NOW | RTLD_LOCAL);
  if (!h) return -1;
  int (*init)(void) = (int (*)(void))dlsym(h, "sodium_init");
  verify_fn f = (verify_fn)dlsym(h, "crypto_sign_verify_detached");
  if (!init || !f || init() < 0) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  pthread_t th[256];
  sjob jobs[256];
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = (sjob){f, pk32, sig64, msg, off, len, n * t / nthreads, n * (t + 1) / nthreads, out};
    pthread_create(&th[t], NULL, srun, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}
