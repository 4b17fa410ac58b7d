/* Dev probe (not product, not a test): OpenSSL 3.0 ChaCha20-Poly1305 seal rate vs threads; modes: 0 re-init per packet, 1 EVP_CipherInit_ex2, 2 no re-init, 3 no re-init and no tag read. */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static int mode; static int npk = 20000; static int ln = 1361;
static void *run(void *arg) {
  (void)arg;
  uint8_t key[32] = {1}, iv[12] = {0};
  uint8_t *in = calloc(ln, 1), *out = malloc(ln + 16);
  EVP_CIPHER *c = mode >= 1 ? EVP_CIPHER_fetch(NULL, "ChaCha20-Poly1305", NULL) : (EVP_CIPHER *)EVP_chacha20_poly1305();
  EVP_CIPHER_CTX *a = EVP_CIPHER_CTX_new();
  EVP_EncryptInit_ex(a, c, NULL, key, NULL);
  for (int i = 0; i < npk; i++) {
    iv[11] = (uint8_t)i; int n;
    if (mode == 1) EVP_CipherInit_ex2(a, NULL, NULL, iv, 1, NULL); else if (mode == 0) EVP_EncryptInit_ex(a, NULL, NULL, NULL, iv); else if (i == 0) EVP_EncryptInit_ex(a, NULL, NULL, NULL, iv);
    EVP_EncryptUpdate(a, NULL, &n, in, 11);
    EVP_EncryptUpdate(a, out + 11, &n, in + 11, ln - 11);
    EVP_EncryptFinal_ex(a, out + ln, &n);
    if (mode != 3) EVP_CIPHER_CTX_ctrl(a, EVP_CTRL_AEAD_GET_TAG, 16, out + ln);
  }
  EVP_CIPHER_CTX_free(a);
  return NULL;
}
int main(int argc, char **argv) {
  mode = atoi(argv[1]); int T = atoi(argv[2]);
  pthread_t th[64]; struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, run, NULL);
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double s = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
  printf("mode %d threads %d: %.2f GiB/s (%.2f per thread)\n", mode, T, (double)T * npk * ln / s / (1 << 30), (double)npk * ln / s / (1 << 30));
}
