/*
 * ossl_quic.c -- CPU timing leg for bench.py --quic: QUIC 1-RTT packet
 * protection (RFC 9001 5.3/5.4) of a batch with OpenSSL's libcrypto (AES-NI /
 * vector code paths), threaded.  TEST/BENCH INFRASTRUCTURE ONLY, like the rest
 * of oracle/: it times what an optimised CPU stack does per packet (quic-go's
 * crypto/aes + GCM assembly is the same class of code); the product path never
 * calls it.  Built by oracle/Makefile into oracle/libossl_quic.so.
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  int suite; /* 0 ChaCha20-Poly1305, 1 AES-128-GCM */
  const uint8_t *key, *iv, *hp, *in;
  const uint64_t *in_off, *out_off, *pn;
  const uint32_t *in_len;
  const uint16_t *pn_offset;
  uint8_t *out;
  uint32_t lo, hi;
  int err;
} job;

static void *run(void *arg) {
  job *j = (job *)arg;
  const int gcm = j->suite == 1;
  EVP_CIPHER_CTX *a = EVP_CIPHER_CTX_new(), *h = EVP_CIPHER_CTX_new();
  const EVP_CIPHER *ac = gcm ? EVP_aes_128_gcm() : EVP_chacha20_poly1305();
  if (!a || !h || EVP_EncryptInit_ex(a, ac, NULL, j->key, NULL) != 1) j->err = 1;
  if (EVP_EncryptInit_ex(h, gcm ? EVP_aes_128_ecb() : EVP_chacha20(), NULL, j->hp, NULL) != 1)
    j->err = 1;
  if (gcm) EVP_CIPHER_CTX_set_padding(h, 0);
  for (uint32_t i = j->lo; i < j->hi && !j->err; i++) {
    const uint8_t *p = j->in + j->in_off[i];
    uint8_t *o = j->out + j->out_off[i];
    const size_t len = j->in_len[i], pno = j->pn_offset[i];
    const size_t pn_len = (size_t)(p[0] & 3) + 1, hdr = pno + pn_len;
    uint8_t nonce[12];
    memcpy(nonce, j->iv, 12);
    for (int k = 0; k < 8; k++) nonce[11 - k] ^= (uint8_t)(j->pn[i] >> (8 * k));
    int n = 0;
    memcpy(o, p, hdr);
    if (EVP_EncryptInit_ex(a, NULL, NULL, NULL, nonce) != 1 ||
        EVP_EncryptUpdate(a, NULL, &n, p, (int)hdr) != 1 ||
        EVP_EncryptUpdate(a, o + hdr, &n, p + hdr, (int)(len - hdr)) != 1 ||
        EVP_EncryptFinal_ex(a, o + len, &n) != 1 ||
        EVP_CIPHER_CTX_ctrl(a, EVP_CTRL_AEAD_GET_TAG, 16, o + len) != 1) {
      j->err = 1;
      break;
    }
    uint8_t mask[64] = {0};
    const uint8_t *sample = o + pno + 4;
    if (gcm) {
      if (EVP_EncryptUpdate(h, mask, &n, sample, 16) != 1) j->err = 1;
    } else {
      static const uint8_t zero[5] = {0};
      if (EVP_EncryptInit_ex(h, NULL, NULL, NULL, sample) != 1 ||
          EVP_EncryptUpdate(h, mask, &n, zero, 5) != 1)
        j->err = 1;
    }
    o[0] ^= mask[0] & ((o[0] & 0x80) ? 0x0f : 0x1f);
    for (size_t k = 0; k < pn_len; k++) o[pno + k] ^= mask[1 + k];
  }
  EVP_CIPHER_CTX_free(a);
  EVP_CIPHER_CTX_free(h);
  return NULL;
}

int ossl_quic_seal_batch(int suite, const uint8_t *key, const uint8_t *iv, const uint8_t *hp,
                         const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                         const uint16_t *pn_offset, const uint64_t *pn, uint32_t n, uint8_t *out,
                         const uint64_t *out_off, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  job *jobs = (job *)calloc((size_t)nthreads, sizeof(job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job jb = {suite, key, iv, hp, in, in_off, out_off, pn, in_len, pn_offset, out,
              (uint32_t)((uint64_t)n * t / nthreads), (uint32_t)((uint64_t)n * (t + 1) / nthreads),
              0};
    jobs[t] = jb;
  }
  for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, run, &jobs[t]);
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  int err = 0;
  for (int t = 0; t < nthreads; t++) err |= jobs[t].err;
  free(jobs);
  free(th);
  return err ? -1 : 0;
}
