/* TEST INFRASTRUCTURE / CPU BASELINE ONLY -- never linked into the product.
 *
 * The CPU baseline SURVEY.md §8(c) and BASELINE.md plan in place of
 * ed25519-dalek's verify_batch (Cargo.lock:668-679; no Rust toolchain or crates
 * in this image): OpenSSL libcrypto EVP_DigestVerify (Ed25519, RFC 8032
 * cofactorless equation, s < L check) over the same SoA batch contract as
 * include/pbft_verify.h, one thread per host core.  Each thread decodes every
 * replica key once (EVP_PKEY per key, the libp2p identity key parse that
 * happens once per peer) and reuses one EVP_MD_CTX.  OpenSSL accepts
 * small-order A/R that dalek verify_strict rejects,
 * so this is a timing baseline on honest rounds, not the parity oracle.
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const uint8_t *keys, *R, *S, *msg;
  const uint16_t *key_idx;
  uint32_t n_keys, msg_len, msg_stride;
  uint64_t lo, hi;
  uint8_t *acc;
  int rc;
} ojob_t;

static void *worker(void *arg) {
  ojob_t *j = (ojob_t *)arg;
  EVP_PKEY **pk = (EVP_PKEY **)calloc(j->n_keys, sizeof(EVP_PKEY *));
  EVP_MD_CTX *ctx = EVP_MD_CTX_new();
  if (!pk || !ctx) { j->rc = -1; goto out; }
  for (uint32_t k = 0; k < j->n_keys; ++k)
    pk[k] = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, j->keys + 32 * (size_t)k, 32);
  uint8_t sig[64];
  for (uint64_t i = j->lo; i < j->hi; ++i) {
    const uint16_t ki = j->key_idx[i];
    if (ki >= j->n_keys || !pk[ki]) { j->acc[i] = 0; continue; }
    memcpy(sig, j->R + 32 * i, 32);
    memcpy(sig + 32, j->S + 32 * i, 32);
    EVP_MD_CTX_reset(ctx);
    int ok = EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, pk[ki]) == 1 &&
             EVP_DigestVerify(ctx, sig, 64, j->msg + (size_t)j->msg_stride * i, j->msg_len) == 1;
    j->acc[i] = (uint8_t)ok;
  }
out:
  if (pk) {
    for (uint32_t k = 0; k < j->n_keys; ++k) EVP_PKEY_free(pk[k]);
    free(pk);
  }
  EVP_MD_CTX_free(ctx);
  return NULL;
}

int ossl_verify_batch(const uint8_t *keys, uint32_t n_keys, const uint8_t *R, const uint8_t *S,
                      const uint16_t *key_idx, const uint8_t *msg, uint32_t msg_len, uint32_t msg_stride, uint64_t N,
                      uint8_t *accept_bytes, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 512) nthreads = 512;
  pthread_t th[512];
  ojob_t jobs[512];
  const uint64_t per = (N + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
  int started = 0, rc = 0;
  for (int t = 0; t < nthreads; ++t) {
    const uint64_t lo = per * (uint64_t)t, hi = lo + per > N ? N : lo + per;
    if (lo >= hi) break;
    jobs[t] = (ojob_t){keys, R, S, msg, key_idx, n_keys, msg_len, msg_stride, lo, hi, accept_bytes, 0};
    if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) { rc = -1; break; }
    ++started;
  }
  for (int t = 0; t < started; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  return rc;
}

/* OpenSSL version string, for the bench line */
const char *ossl_version(void) { return OpenSSL_version(OPENSSL_VERSION); }
