/*
 * zt_oracle.h -- CPU restatement of ExaGraphica/zlib.ts's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * engine in zlib.ts_amd/ and the "port" CPU baseline timed by bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (libzt.so, the N-API addon, the JS facade) never links or calls
 * it.
 *
 * Pinned against the reference: the vectors in tests/golden were produced by running
 * the reference's own compiled JS (/root/reference/js) under Node
 * (tools/gen_golden.mjs); tests/test_oracle_golden.py checks every function
 * below against those vectors.
 *
 * Every function mirrors the reference bit for bit, quirks included
 * (Uint16 heap truncation, lazy>0 end-of-input duplication, over-strict
 * readBits EOF check, typed-array out-of-range semantics).
 */
#ifndef ZT_ORACLE_H
#define ZT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (negative = the reference threw) */
#define ZO_OK 0
#define ZO_ERR_INVALID_COMPRESSION_TYPE -1 /* src/RawDeflate.ts:110 'invalid compression type' */
#define ZO_ERR_INVALID_INDEX -2            /* src/Bitstream.ts:29 Error('invalid index')      */
#define ZO_ERR_TYPE -3                     /* a JS TypeError the reference would raise         */
#define ZO_ERR_INFLATE -10                 /* an Error thrown by src/RawInflate.ts; see msg    */

/* src/CRC32.ts:25-47  CRC32.update(data, crc) over data[0..n) */
uint32_t zo_crc32_update(const uint8_t *data, size_t n, uint32_t crc);
/* src/CRC32.ts:54-56  CRC32.single(num, crc) */
uint32_t zo_crc32_single(uint32_t num, uint32_t crc);
/* src/Adler32.ts:28-48  Adler32.update(adler, array, n) */
uint32_t zo_adler32_update(uint32_t adler, const uint8_t *data, size_t n);

/*
 * src/RawDeflate.ts:67-114  new RawDeflate(input, opts).compress()
 *   lazy, ctype       -- opts.lazy / opts.compressionType (0 NONE, 1 FIXED, 2 DYNAMIC)
 *   outbuf/outbuf_len -- opts.outputBuffer (NULL => fresh Uint8Array(0x8000))
 *   out_index         -- opts.outputIndex
 * On success *out (malloc'd, free with zo_free) holds the returned Uint8Array
 * (bytes [0, *out_len)), and *op the object's .op afterwards.
 */
int zo_raw_deflate(const uint8_t *in, size_t n, int lazy, int ctype,
                   const uint8_t *outbuf, size_t outbuf_len, size_t out_index,
                   uint8_t **out, size_t *out_len, size_t *op);

/*
 * src/RawInflate.ts:104-140  new RawInflate(input, {index, bufferSize,
 * bufferType, resize}).decompress().  On success (*out, *out_len) is the returned
 * array and *ip the object's .ip.  On ZO_ERR_INFLATE, msg holds the Error text.
 */
int zo_raw_inflate(const uint8_t *in, size_t n, size_t index, int buffer_type,
                   size_t buffer_size, uint8_t **out, size_t *out_len,
                   size_t *ip, char *msg, size_t msg_cap);

/* Token-level view of src/LZ77.ts:196-283 for tests: returns the Uint16
 * token array (malloc'd) and the lit/len + dist histograms. */
int zo_lz77_encode(const uint8_t *in, size_t n, int lazy, uint16_t **tokens,
                   size_t *ntokens, uint32_t freqs_litlen[286],
                   uint32_t freqs_dist[30]);

/* src/RawDeflate.ts:440-474 getLengths(freqs, limit) */
int zo_huffman_lengths(const uint32_t *freqs, size_t nsym, int limit,
                       uint8_t *lengths);

/* Test-data generators (not reference functions): kind 0 xorshift32,
 * 1 wordsalad, 2 structured; see tools/gen_golden.mjs. */
void zo_gen(int kind, uint32_t seed, uint8_t *out, size_t n);

void zo_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
