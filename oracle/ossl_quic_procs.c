/*
 * ossl_quic_procs.c -- CPU timing leg for bench.py --quic, in PROCESSES:
 * OpenSSL 3.0's EVP layer serialises threads on its per-call bookkeeping
 * (measured on the GPU box: 16 threads 6.1 GiB/s, 16 processes 24.9 GiB/s
 * for the same ChaCha20-Poly1305 loop; scripts/dev/ossl_*.c), so the fair
 * multi-core CPU rate of quic-go-class code is P independent processes.
 * TEST/BENCH INFRASTRUCTURE ONLY (oracle/): it seals with ossl_quic.c's
 * per-packet routine and never touches a GPU.  bench.py starts it as a
 * child process.
 *
 * usage: ossl_quic_procs SUITE PROCS PACKETS LEN SECONDS
 * prints one JSON line: aggregate and per-process GiB/s of payload sealed.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

int ossl_quic_seal_batch(int suite, const uint8_t *key, const uint8_t *iv, const uint8_t *hp,
                         const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                         const uint16_t *pn_offset, const uint64_t *pn, uint32_t n, uint8_t *out,
                         const uint64_t *out_off, int nthreads);

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s SUITE PROCS PACKETS LEN SECONDS\n", argv[0]);
    return 2;
  }
  const int suite = atoi(argv[1]), P = atoi(argv[2]);
  const uint32_t m = (uint32_t)atoi(argv[3]), ln = (uint32_t)atoi(argv[4]);
  const double secs = atof(argv[5]);
  if (P < 1 || P > 256 || m == 0 || ln < 32) return 2;
  double *res = mmap(NULL, sizeof(double) * 2 * P, PROT_READ | PROT_WRITE,
                     MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (res == MAP_FAILED) return 1;
  for (int w = 0; w < P; w++) {
    if (fork() == 0) {
      uint8_t key[32], iv[12], hp[32];
      for (int i = 0; i < 32; i++) key[i] = (uint8_t)(i * 7 + 1), hp[i] = (uint8_t)(i * 5 + 3);
      for (int i = 0; i < 12; i++) iv[i] = (uint8_t)(i * 3);
      uint8_t *in = malloc((size_t)m * ln), *out = malloc((size_t)m * (ln + 16));
      uint64_t *ioff = malloc(8ull * m), *ooff = malloc(8ull * m), *pn = malloc(8ull * m);
      uint32_t *len = malloc(4ull * m);
      uint16_t *pno = malloc(2ull * m);
      for (uint32_t i = 0; i < m; i++) {
        ioff[i] = (uint64_t)i * ln;
        ooff[i] = (uint64_t)i * (ln + 16);
        len[i] = ln;
        pno[i] = 9;
        pn[i] = i;
        uint8_t *p = in + ioff[i];
        for (uint32_t k = 0; k < ln; k++) p[k] = (uint8_t)(k * 13 + i);
        p[0] = 0x41;  // short header, 2-byte packet number
      }
      long reps = 0;
      const double t0 = now();
      double t1 = t0;
      while (reps < 1 || t1 - t0 < secs) {
        if (ossl_quic_seal_batch(suite, key, iv, hp, in, ioff, len, pno, pn, m, out, ooff, 1))
          _exit(1);
        reps++;
        t1 = now();
      }
      res[2 * w] = (double)reps * m * ln;
      res[2 * w + 1] = t1 - t0;
      _exit(0);
    }
  }
  int bad = 0;
  for (int w = 0; w < P; w++) {
    int st = 0;
    wait(&st);
    bad |= !WIFEXITED(st) || WEXITSTATUS(st) != 0;
  }
  if (bad) return 1;
  double bytes = 0, tmax = 0, per_min = 1e30, per_max = 0;
  for (int w = 0; w < P; w++) {
    bytes += res[2 * w];
    if (res[2 * w + 1] > tmax) tmax = res[2 * w + 1];
    const double r = res[2 * w] / res[2 * w + 1] / (1 << 30);
    if (r < per_min) per_min = r;
    if (r > per_max) per_max = r;
  }
  printf("{\"suite\": %d, \"procs\": %d, \"gib_s\": %.3f, \"per_proc_gib_s_min\": %.3f, "
         "\"per_proc_gib_s_max\": %.3f, \"packets\": %u, \"len\": %u}\n",
         suite, P, bytes / tmax / (1 << 30), per_min, per_max, m, ln);
  return 0;
}
