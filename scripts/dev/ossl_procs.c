/* Dev probe (not product, not a test): the same OpenSSL seal loop in forked processes. */
#include <openssl/evp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>
int main(int argc, char **argv) {
  int T = atoi(argv[1]), npk = 20000, ln = 1361;
  struct timespec t0, t1; clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < T; t++) if (fork() == 0) {
    uint8_t key[32] = {1}, iv[12] = {0};
    uint8_t *in = calloc(ln, 1), *out = malloc(ln + 16);
    EVP_CIPHER_CTX *a = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(a, EVP_chacha20_poly1305(), NULL, key, NULL);
    for (int i = 0; i < npk; i++) { int n; iv[11] = i;
      EVP_EncryptInit_ex(a, NULL, NULL, NULL, iv);
      EVP_EncryptUpdate(a, NULL, &n, in, 11); EVP_EncryptUpdate(a, out + 11, &n, in + 11, ln - 11);
      EVP_EncryptFinal_ex(a, out + ln, &n); EVP_CIPHER_CTX_ctrl(a, EVP_CTRL_AEAD_GET_TAG, 16, out + ln); }
    _exit(0);
  }
  for (int t = 0; t < T; t++) wait(NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  double s = (t1.tv_sec - t0.tv_sec) + (t1.tv_nsec - t0.tv_nsec) * 1e-9;
  printf("procs %d: %.2f GiB/s\n", T, (double)T * npk * ln / s / (1 << 30));
}
