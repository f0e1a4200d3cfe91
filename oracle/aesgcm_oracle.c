/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Nothing in the product path
 * (uplink_amd/, include/) may link, load or call this file.  Only tests/ and
 * the CPU-baseline legs of the benches use it.
 *
 * CPU restatement of storj/uplink's segment encryption:
 *
 *   nonceForPosition / deriveContentNonce   splitter/common.go:27-32, streams/store.go:264-270
 *       24-byte storj.Nonce, zero, incremented (little-endian) by
 *       PartNumber<<32 | (Index+1)
 *   encryption.NewEncrypter(EncAESGCM, &contentKey, &nonce, BlockSize)
 *                                            splitter/splitter.go:156 (BlockSize = 29*256, project.go:84)
 *   encryption.TransformWriterPadded         splitter/splitter.go:170
 *   encryption.NewDecrypter / Transform / Unpad   streams/store.go:347-382
 *
 * The cipher code is storj.io/common/encryption (go.mod:14), not vendored and
 * absent here.  Its published behaviour, restated: AES-256-GCM over blocks of
 * InBlockSize = BlockSize - 16 plaintext bytes; block b is sealed with the
 * 12-byte nonce = first 12 bytes of the starting nonce incremented
 * (little-endian, with carry) by b, no additional data, and written as
 * ciphertext || 16-byte tag (OutBlockSize = BlockSize).  The plaintext is
 * padded to a multiple of InBlockSize with the PadReader rule (SURVEY.md
 * Appendix B).  A block that fails authentication makes the decrypter fail.
 *
 * The AES-256-GCM primitive is OpenSSL's (libcrypto.so.3 in this image), the
 * same standard cipher as Go's crypto/aes + crypto/cipher that
 * storj.io/common uses.  It is pinned against the GCM specification's test
 * cases 13-15 (tests/golden/aesgcm_vectors.json, tests/test_aesgcm.py).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>

/* encryption.incrementBytes: little-endian add with carry; returns 1 when the
 * amount did not fit (the reference reports that as truncation) */
int ag_increment(uint8_t *buf, size_t len, uint64_t amount) {
    for (size_t i = 0; i < len && amount; i++) {
        uint64_t sum = (uint64_t)buf[i] + (amount & 0xFF);
        buf[i] = (uint8_t)sum;
        amount = (amount >> 8) + (sum >> 8);
    }
    return amount != 0;
}

/* one GCM seal: out = ciphertext (len bytes) || tag (16 bytes) */
int ag_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len, const uint8_t *in,
            size_t len, uint8_t *out) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int ok = c && EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, NULL, NULL) &&
             EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, NULL) &&
             EVP_EncryptInit_ex(c, NULL, NULL, key, nonce);
    int n = 0, f = 0;
    if (ok && aad_len) ok = EVP_EncryptUpdate(c, NULL, &n, aad, (int)aad_len);
    if (ok && len) ok = EVP_EncryptUpdate(c, out, &n, in, (int)len);
    if (ok) ok = EVP_EncryptFinal_ex(c, out + n, &f);
    if (ok) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out + len);
    EVP_CIPHER_CTX_free(c);
    return ok ? 0 : -1;
}

/* one GCM open of in = ciphertext (len bytes) || tag; 0 = authentic */
int ag_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *in, size_t len, uint8_t *out) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int n = 0, f = 0;
    int ok = c && EVP_DecryptInit_ex(c, EVP_aes_256_gcm(), NULL, NULL, NULL) &&
             EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, NULL) &&
             EVP_DecryptInit_ex(c, NULL, NULL, key, nonce);
    if (ok && len) ok = EVP_DecryptUpdate(c, out, &n, in, (int)len);
    if (ok) ok = EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, (void *)(in + len));
    if (ok) ok = EVP_DecryptFinal_ex(c, out + n, &f) > 0;
    EVP_CIPHER_CTX_free(c);
    return ok ? 0 : -1;
}

typedef struct {
    const uint8_t *key, *nonce, *in;
    uint8_t *out;
    size_t in_block, first, count;
    int open, failed;
    int64_t first_bad;
} ag_job;

/* one AEAD per worker, as the reference keeps one cipher.AEAD per segment
 * (NewAESGCMEncrypter); per block only the nonce changes */
static void *ag_worker(void *a) {
    ag_job *j = (ag_job *)a;
    const size_t ob = j->in_block + 16;
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int ok = c && (j->open ? EVP_DecryptInit_ex(c, EVP_aes_256_gcm(), NULL, NULL, NULL)
                           : EVP_EncryptInit_ex(c, EVP_aes_256_gcm(), NULL, NULL, NULL)) &&
             EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_IVLEN, 12, NULL) &&
             (j->open ? EVP_DecryptInit_ex(c, NULL, NULL, j->key, NULL) : EVP_EncryptInit_ex(c, NULL, NULL, j->key, NULL));
    for (size_t b = j->first; ok && b < j->first + j->count; b++) {
        uint8_t nonce[12];
        memcpy(nonce, j->nonce, 12);
        ag_increment(nonce, 12, b);
        int n = 0, f = 0, good;
        if (j->open) {
            const uint8_t *in = j->in + b * ob;
            uint8_t *out = j->out + b * j->in_block;
            good = EVP_DecryptInit_ex(c, NULL, NULL, NULL, nonce) && EVP_DecryptUpdate(c, out, &n, in, (int)j->in_block) &&
                   EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, 16, (void *)(in + j->in_block)) &&
                   EVP_DecryptFinal_ex(c, out + n, &f) > 0;
        } else {
            const uint8_t *in = j->in + b * j->in_block;
            uint8_t *out = j->out + b * ob;
            good = EVP_EncryptInit_ex(c, NULL, NULL, NULL, nonce) && EVP_EncryptUpdate(c, out, &n, in, (int)j->in_block) &&
                   EVP_EncryptFinal_ex(c, out + n, &f) && EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, out + j->in_block);
        }
        if (!good && !j->failed) {
            j->failed = 1;
            j->first_bad = (int64_t)b;
        }
    }
    if (!ok && !j->failed) {
        j->failed = 1;
        j->first_bad = (int64_t)j->first;
    }
    EVP_CIPHER_CTX_free(c);
    return NULL;
}

static int64_t ag_run(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *in, size_t nblocks,
                      size_t in_block, uint8_t *out, int threads, int open) {
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if ((size_t)threads > nblocks) threads = nblocks ? (int)nblocks : 1;
    pthread_t th[64];
    ag_job jobs[64];
    size_t per = nblocks / threads, extra = nblocks % threads, first = 0;
    for (int t = 0; t < threads; t++) {
        jobs[t] = (ag_job){key, nonce, in, out, in_block, first, per + ((size_t)t < extra), open, 0, -1};
        first += jobs[t].count;
        if (t < threads - 1) pthread_create(&th[t], NULL, ag_worker, &jobs[t]);
    }
    ag_worker(&jobs[threads - 1]);
    for (int t = 0; t < threads - 1; t++) pthread_join(th[t], NULL);
    int64_t bad = -1;
    for (int t = 0; t < threads; t++)
        if (jobs[t].failed && (bad < 0 || jobs[t].first_bad < bad)) bad = jobs[t].first_bad;
    return bad;
}

/* Encrypter.Transform over nblocks padded plaintext blocks of in_block bytes
 * (block b with nonce + b); out: nblocks * (in_block + 16).  Returns -1 on
 * success, else the first block that failed. */
int64_t ag_encrypt_blocks(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *plain, size_t nblocks,
                          size_t in_block, uint8_t *out, int threads) {
    return ag_run(key, nonce, plain, nblocks, in_block, out, threads, 0);
}

/* Decrypter.Transform: returns -1 when every block authenticates, else the
 * first block that did not */
int64_t ag_decrypt_blocks(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *cipher, size_t nblocks,
                          size_t in_block, uint8_t *out, int threads) {
    return ag_run(key, nonce, cipher, nblocks, in_block, out, threads, 1);
}
