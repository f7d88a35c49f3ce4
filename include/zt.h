/*
 * zt.h -- C-ABI of the MI355X-native DEFLATE engine (libzt.so).
 *
 * Drop-in boundary for ExaGraphica/zlib.ts's hot path.  Every entry point is
 * plain C (pointers + sizes, no torch/HIP types), synchronous, and computes on
 * the GPU; there is no CPU fallback -- without a usable HIP device the calls
 * return ZT_E_NO_DEVICE.  The N-API addon (zlib.ts_amd/native/zt_napi.cc)
 * binds these for the JS facade that keeps the reference's class shapes.
 *
 * Each function names the reference interface it replaces (path:line in
 * ExaGraphica/zlib.ts @ 2024-10-08).  Error codes map 1:1 onto the
 * reference's thrown messages; zt_last_error_message() returns the exact text.
 */
#ifndef ZT_H
#define ZT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define ZT_OK 0
#define ZT_E_INVALID_COMPRESSION_TYPE -1 /* 'invalid compression type'  src/RawDeflate.ts:110 */
#define ZT_E_INVALID_INDEX -2            /* Error('invalid index')      src/Bitstream.ts:29   */
#define ZT_E_INPUT_BROKEN -10            /* 'input buffer is broken'    src/RawInflate.ts:188,282 */
#define ZT_E_INVALID_CODE_LENGTH -11     /* 'invalid code length: N'    src/RawInflate.ts:238 */
#define ZT_E_UNKNOWN_BTYPE -12           /* 'unknown BTYPE: N'          src/RawInflate.ts:168 */
#define ZT_E_STORED_LEN -13              /* '...uncompressed block header: LEN'  :266 */
#define ZT_E_STORED_NLEN -14             /* '...uncompressed block header: NLEN' :272 */
#define ZT_E_INVALID_DISTANCE -15        /* RFC 1951 violation the reference does not check (:507) */
#define ZT_E_INVALID_SYMBOL -16          /* lit/len 286-287 or dist 30-31 used (RFC 1951 3.2.6) */
#define ZT_E_BAD_TREE -17                /* over-subscribed / empty code-length set */
/* containers */
#define ZT_E_GZIP_SIGNATURE -30          /* Error('invalid file signature:ID1,ID2')  src/GUnzip.ts:77 */
#define ZT_E_GZIP_METHOD -31             /* Error('unknown compression method: CM')  src/GUnzip.ts:82 */
#define ZT_E_GZIP_HCRC -32               /* Error('invalid header crc16')            src/GUnzip.ts:130 */
#define ZT_E_GZIP_CRC32 -33              /* Error('invalid CRC-32 checksum: 0x.. / 0x..') src/GUnzip.ts:162 */
#define ZT_E_GZIP_ISIZE -34              /* Error('invalid input size: N / M')       src/GUnzip.ts:169 */
#define ZT_E_ZLIB_METHOD -40             /* Error('unsupported compression method')  src/Inflate.ts:47 */
#define ZT_E_ZLIB_FCHECK -41             /* Error('invalid fcheck flag:N')           src/Inflate.ts:52 */
#define ZT_E_ZLIB_FDICT -42              /* Error('fdict flag is not supported')     src/Inflate.ts:57 */
#define ZT_E_ZLIB_ADLER -43              /* Error('invalid adler-32 checksum')       src/Inflate.ts:88 */
#define ZT_E_ZIP_FORMAT -50              /* Error('End of Central Directory Record not found' | 'invalid file
                                            header signature' | 'invalid file header size' | 'invalid local
                                            file header signature')  src/Unzip.ts:39,89,160,236 */
#define ZT_E_ZIP_CRC -51                 /* Error('Incorrect crc: file=0x.., data=0x..')  src/Unzip.ts:296 */
#define ZT_E_ZIP_ENCRYPTED -52           /* Error('encrypted: please set password')  src/Unzip.ts:266 (no ZipCrypto) */
#define ZT_E_NO_DEVICE -100              /* no HIP device: the engine never falls back to the CPU */
#define ZT_E_HIP -101                    /* HIP runtime failure (see message) */
#define ZT_E_NOMEM -102
#define ZT_E_ARG -103
#define ZT_E_INTERNAL -104               /* engine invariant broken (see message) */

/* ---- devices ----------------------------------------------------------- */
int zt_device_count(void);
/* Select the device used by the calling thread (default 0). */
int zt_set_device(int device);
/* Devices the batch calls (zt_*_batch) split their buffers over: bit d =
 * device d (config C4: one node's GPUs, no collective -- every buffer is
 * independent).  0 restores the default: the calling thread's device. */
int zt_set_devices(uint64_t mask);
/* Text of the last error on this thread, formatted like the reference's
 * message (e.g. "invalid code length: 9"). */
const char *zt_last_error_message(void);
/* Library version string. */
const char *zt_version(void);
/* Free a buffer returned by the library (every output pointer, batch items
 * included; never free() them directly: batch items share allocations, and
 * outputs of 8 MiB or more return to a bounded host output pool -- reused,
 * registered with HIP, by the next output of a similar size; at most
 * ZT_HOST_POOL_MB free MiB kept (default 4096, 0: no pool);
 * zt_release_scratch drops them). */
void zt_free(void *p);

/* ---- checksums (host pointers) ------------------------------------------ */
/* Replaces CRC32.update(data, crc, pos, length)  src/CRC32.ts:25-47 (and
 * CRC32.create, :13-15, with crc = 0).  Result in *out (unsigned, >>> 0). */
int zt_crc32_update(uint32_t crc, const uint8_t *data, size_t len, uint32_t *out);
/* Replaces Adler32.update(adler, array, len, pos)  src/Adler32.ts:28-48 (and
 * Adler32.create, :13-20, with adler = 1). */
int zt_adler32_update(uint32_t adler, const uint8_t *data, size_t len, uint32_t *out);
/* Both checksums in one read of the data (the GZip/Zip/zlib containers call
 * CRC32/Adler32 beside RawDeflate: src/GZip.ts:180, src/Deflate.ts:81). */
int zt_checksums(const uint8_t *data, size_t len, uint32_t crc_in, uint32_t adler_in, uint32_t *crc_out,
                 uint32_t *adler_out);

/* ---- raw DEFLATE (RFC 1951) ---------------------------------------------- */
typedef struct {
  int compression_type; /* RawDeflateOptions.compressionType: 0 NONE, 1 FIXED, 2 DYNAMIC (default 2) */
  int lazy;             /* RawDeflateOptions.lazy (reference semantics: defer matches shorter than this) */
  int level;            /* engine extension: 1..9, 0 = store; default (-1) = 6 */
} zt_deflate_opts;

/* Replaces new RawDeflate(input, opts).compress()  src/RawDeflate.ts:67-114.
 * *out (free with zt_free) receives a complete raw DEFLATE stream of *out_len
 * bytes: a valid RFC 1951 stream that the reference RawInflate decodes to
 * `in` bit-exactly.  (The outputBuffer/outputIndex prefix handling of the
 * reference lives in the facade.)  opts may be NULL. */
int zt_deflate_raw(const uint8_t *in, size_t n, const zt_deflate_opts *opts, uint8_t **out, size_t *out_len);

typedef struct {
  int buffer_type; /* RawInflateOptions.bufferType (0 BLOCK, 1 ADAPTIVE); accepted, output identical */
  size_t buffer_size; /* RawInflateOptions.bufferSize; accepted (capacity is not observable) */
  int ref_strict;  /* 1: also fail where the reference's over-strict readBits EOF check
                      (src/RawInflate.ts:187) throws 'input buffer is broken' on a valid stream */
} zt_inflate_opts;

/* Replaces new RawInflate(input, {index}).decompress()  src/RawInflate.ts:104-140.
 * Decodes the stream that starts at in[index].  *end_ip receives the
 * reference's .ip after decompress (byte just past the last used bit).
 * opts may be NULL. */
int zt_inflate_raw(const uint8_t *in, size_t n, size_t index, const zt_inflate_opts *opts, uint8_t **out,
                   size_t *out_len, size_t *end_ip);

/* Replaces RawInflateStream.decompress(input, ip)  src/RawInflateStream.ts:67-120
 * (SURVEY.md 8(f) row 4): resumable decode of a stream that arrives in
 * pieces.  Decodes from bit `bit_pos` of in[0..n) (bit k = bit k % 8 of byte
 * k / 8), with window[0..wlen) -- the output already produced, of which the
 * last 32 KiB are used -- as match history, every block that lies completely
 * inside the input.  *out receives those blocks' bytes, *end_bits the bit
 * position just after the last of them (resume there with more input),
 * *finished 1 once the BFINAL block was decoded.  Running out of input is not
 * an error (the output then ends at the last complete block); a corrupt
 * stream fails with the reference's message (an error within the last 8
 * bytes of the input counts as running out of input until more arrives).  The reference resumes at
 * symbol granularity; this engine at block granularity: the concatenated
 * output is identical. */
int zt_inflate_raw_resume(const uint8_t *in, size_t n, uint64_t bit_pos, const uint8_t *window, size_t wlen,
                          uint8_t **out, size_t *out_len, uint64_t *end_bits, int *finished);
/* The same for the last piece of a stream (no more input will come): every
 * error is reported as-is -- a stream that is corrupt near its end, or ends
 * before its BFINAL block, fails with the reference's message instead of
 * waiting for more input (RawInflateStream.finish() in the JS / Python
 * facades). */
int zt_inflate_raw_resume_final(const uint8_t *in, size_t n, uint64_t bit_pos, const uint8_t *window, size_t wlen,
                                uint8_t **out, size_t *out_len, uint64_t *end_bits, int *finished);

/* Batch forms: `count` independent buffers in one launch (config C2/C4).
 * status[i] receives each item's code; the call returns the first failure. */
int zt_inflate_raw_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_inflate_opts *opts,
                         uint8_t **out, size_t *out_len, size_t *end_ip, int *status);
int zt_deflate_raw_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_deflate_opts *opts,
                         uint8_t **out, size_t *out_len, int *status);

/* ---- containers: GZip (RFC 1952) and zlib (RFC 1950) ---------------------- */
/* The input is uploaded once; the deflate pipeline and the CRC-32 / Adler-32
 * kernel both read that device copy (the reference deflates, then walks the
 * input again for the checksum: src/GZip.ts:163-180, src/Deflate.ts:81-85). */
typedef struct {
  zt_deflate_opts deflate; /* GZipOptions.deflateOptions */
  int fname;               /* FNAME: name[0..name_len) is written (GZipOptions.filename) */
  int fcomment;            /* FCOMMENT: comment[0..comment_len) (GZipOptions.comment) */
  int fhcrc;               /* FHCRC (GZipOptions.hcrc) */
  uint32_t mtime;          /* MTIME (the reference writes floor(Date.now()/1000)) */
  const uint8_t *name;     /* header bytes, already encoded as the reference does */
  size_t name_len;         /* (charCode <= 0xFF: one byte, else two LE bytes: src/GZip.ts:133-140) */
  const uint8_t *comment;
  size_t comment_len;
} zt_gzip_opts;

/* Replaces new GZip(input, opts).compress()  src/GZip.ts:96-194: one member,
 * header + raw DEFLATE + CRC-32 + ISIZE.  *crc_out (may be NULL) = GZip.crc32. */
int zt_gzip_compress(const uint8_t *in, size_t n, const zt_gzip_opts *opts, uint8_t **out, size_t *out_len,
                     uint32_t *crc_out);

/* Batch GZip (config C4): `count` independent members, each as
 * zt_gzip_compress makes it (the same opts for all), in one pipeline per
 * device: the buffers are packed at 32 KiB boundaries and uploaded once, the
 * batch deflate pipeline and the batched CRC-32 kernels read the same device
 * bytes, and the devices of zt_set_devices share the batch (largest buffers
 * first onto the least loaded device).  out[i] is library memory: release
 * each with zt_free (the outputs of one call may share one allocation, which
 * goes with its last item).
 * Replaces a loop of new GZip(in[i], opts).compress()  src/GZip.ts:96-194. */
int zt_gzip_compress_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_gzip_opts *opts,
                           uint8_t **out, size_t *out_len, int *status);
/* The same for zlib streams: a loop of new Deflate(in[i], opts).compress()
 * src/Deflate.ts:60-99 (CMF/FLG, raw DEFLATE, Adler-32). */
int zt_zlib_compress_batch(const uint8_t *const *in, const size_t *n, size_t count, const zt_deflate_opts *opts,
                           uint8_t **out, size_t *out_len, int *status);

/* CRC-32 (initial 0) of `count` host buffers in one batched kernel launch
 * (CRC32.create per buffer, src/CRC32.ts:25-47). */
int zt_crc32_batch(const uint8_t *const *in, const size_t *n, size_t count, uint32_t *crc_out);

/* ---- Zip / Unzip (no ZipCrypto) ---------------------- */
/* One Zip.addFile(input, filename, opts) (src/Zip.ts:80-108). */
typedef struct {
  const uint8_t *name;    /* filename bytes (stringToByteArray: charCode & 0xFF) */
  size_t name_len;
  const uint8_t *comment; /* file comment bytes, or NULL */
  size_t comment_len;
  int method;             /* ZipCompressionMethod: 8 DEFLATE (default), 0 STORE */
  int os;                 /* ZipOperatingSystem of the central header (default MSDOS = 0) */
  uint8_t mtime[4];       /* DOS time / date bytes exactly as src/Zip.ts:130-139 builds them */
  zt_deflate_opts deflate;/* deflateOptions */
} zt_zip_file;
/* Replaces Zip.compress()  src/Zip.ts:117-372: local headers + data, central
 * directory, end record, laid out as the reference does; all DEFLATE members
 * in one batch pipeline, all CRC-32s batched on the device.  The reference's
 * extraField (written with a zero length, src/Zip.ts:215) is not supported. */
int zt_zip_compress(const uint8_t *const *in, const size_t *n, const zt_zip_file *files, size_t count,
                    const uint8_t *comment, size_t comment_len, uint8_t **out, size_t *out_len);
/* One entry of an archive (FileHeader + its data, src/Unzip.ts:64-130). */
typedef struct {
  size_t name_off, name_len;       /* filename bytes in the input */
  size_t comment_off, comment_len; /* file comment bytes in the input */
  size_t data_off, data_len;       /* decompressed data in the output */
  size_t local_offset;             /* relative offset of the local header */
  uint32_t version, os, need_version, flags, method, time, date;
  uint32_t crc32, compressed_size, plain_size; /* central directory fields */
  uint32_t local_crc32, local_method;          /* local header fields (what getFileData uses) */
  uint32_t data_crc32;             /* CRC-32 of the decompressed data (computed on the GPU) */
  int32_t status;                  /* 0, or what getFileData(i) throws; message in `message` */
  char message[96];
} zt_unzip_entry;
/* Replaces new Unzip(input, {verify}) + getFilenames() + getFileData(i) for
 * every i  src/Unzip.ts:150-342: the archive's entries are parsed with the
 * reference's checks and inflated in one batch.  Archive-level errors return
 * with nothing filled; otherwise *out (all entries' data) and *entries are
 * filled and the first failing entry's status is returned (its message set). */
int zt_unzip(const uint8_t *in, size_t n, int verify, uint8_t **out, size_t *out_len, zt_unzip_entry **entries,
             size_t *count);

/* One decoded member (GUnzipMember, src/GUnzip.ts:66-175).  Offsets index the
 * input buffer (name, comment) or the concatenated output (data). */
typedef struct {
  uint32_t flg, mtime, xfl, os, xlen;
  size_t name_off, name_len;       /* valid when flg & FNAME */
  size_t comment_off, comment_len; /* valid when flg & FCOMMENT */
  uint32_t has_crc16, crc16;
  uint32_t crc32, isize;
  size_t data_off, data_len;
} zt_gzip_member;

/* Replaces new GUnzip(input).decompress() + getMembers()  src/GUnzip.ts:53-63:
 * every member until the input is consumed, their outputs concatenated.
 * *members (free with zt_free; may be NULL) receives *nmembers entries. */
int zt_gunzip(const uint8_t *in, size_t n, uint8_t **out, size_t *out_len, zt_gzip_member **members,
              size_t *nmembers);

/* Replaces new Deflate(input, {compressionType, lazy}).compress()
 * src/Deflate.ts:60-99: CMF/FLG (FLEVEL = compressionType) + raw DEFLATE +
 * Adler-32 big-endian.  *adler_out (may be NULL) = Deflate.adler32. */
int zt_zlib_compress(const uint8_t *in, size_t n, const zt_deflate_opts *opts, uint8_t **out, size_t *out_len,
                     uint32_t *adler_out);

/* Replaces new Inflate(input, {index, verify}).decompress()  src/Inflate.ts:34-93.
 * *end_ip = Inflate.ip (just past the DEFLATE stream, before the Adler-32). */
int zt_zlib_decompress(const uint8_t *in, size_t n, size_t index, int verify, uint8_t **out, size_t *out_len,
                       size_t *end_ip, uint32_t *adler_out);

/* ---- device-resident forms (inputs already in HBM; used by bench.py) ------ */
/* `stream` is a hipStream_t (NULL = the library's stream for this device).
 * Pointers are device pointers of the current device.  They enqueue work and
 * return; results written to device memory are valid after the stream syncs,
 * host outputs (sizes) are valid on return. */
int zt_dev_checksums(const void *d_in, size_t n, uint32_t crc_in, uint32_t adler_in, uint32_t *crc_out,
                     uint32_t *adler_out, void *stream);

typedef struct zt_deflate_plan zt_deflate_plan;
/* Workspace for deflating up to max_n bytes (chunk scratch, token buffers). */
int zt_deflate_plan_create(size_t max_n, const zt_deflate_opts *opts, zt_deflate_plan **plan);
void zt_deflate_plan_destroy(zt_deflate_plan *plan);
/* Upper bound on the compressed size of n bytes. */
size_t zt_deflate_bound(size_t n);
/* Deflate d_in[0..n) into d_out (capacity zt_deflate_bound(n)); writes the
 * stream length to *out_len (host).  When final == 0 the stream is left open
 * (ends on a byte-aligned sync point, no BFINAL) so shards can be
 * concatenated; `halo` bytes before d_in (d_in - halo .. d_in) are used as
 * the match window of the first chunk (multi-GPU shards). */
int zt_deflate_dev(zt_deflate_plan *plan, const void *d_in, size_t n, size_t halo, int final, void *d_out,
                   size_t *out_len, void *stream);

typedef struct zt_inflate_plan zt_inflate_plan;
int zt_inflate_plan_create(size_t max_in, size_t max_out, zt_inflate_plan **plan);
void zt_inflate_plan_destroy(zt_inflate_plan *plan);
/* Inflate the raw stream d_in[0..n) into d_out (capacity out_cap).  Streams
 * carrying sync / restart points (empty stored blocks, which zt_deflate_dev
 * writes after every block and every 1 MiB of input) are decoded
 * segment-parallel (inflate_seg.hip + inflate_tok.hip); any other stream --
 * the reference's own single-block output, zlib / gzip streams -- by the
 * general speculative decoder (inflate_gen.hip); a stream neither path
 * finishes (a corrupt one) by one wavefront, which reports the reference's
 * exact error.  Results are identical whichever path decodes. */
int zt_inflate_dev(zt_inflate_plan *plan, const void *d_in, size_t n, void *d_out, size_t out_cap,
                   size_t *out_len, size_t *end_ip, void *stream);

/* ---- benchmark / test support (no reference counterpart) ---- */
/* Synthetic corpus: 64 KiB piece i is generator `kind`
 * (0 xorshift32, 1 wordsalad, 2 structured int32 deltas, 3 mixed per 4 MiB
 * window) seeded with seed + i.  d_out must be 4-byte aligned.  With a
 * null stream the call returns when the data is written. */
int zt_synth_dev(int kind, uint32_t seed, void *d_out, size_t n, void *stream);
/* The same corpus from piece `piece0` on: bytes [piece0 * 65536, piece0 *
 * 65536 + n) of the whole corpus (one rank's shard of a sharded buffer,
 * config C3), so every rank generates exactly its slice. */
int zt_synth_dev_at(int kind, uint32_t seed, uint64_t piece0, void *d_out, size_t n, void *stream);
/* Kernel-time accounting with HIP events on the launch stream: the deflate
 * match-finding kernel (the dominant one), the whole deflate kernel pipeline,
 * and the inflate decode kernel of the device paths. */
typedef struct {
  double deflate_ms; /* match_kernel */
  uint64_t deflate_launches;
  double inflate_ms; /* inflate decode kernels (two-phase: tokenize + resolve; else the one-wave decode) */
  uint64_t inflate_launches;
  double deflate_pipeline_ms; /* match .. gather */
  uint64_t deflate_pipelines;
  double inflate_tok_ms; /* two-phase inflate: phase A (tokenize_kernel) alone */
  uint64_t inflate_toks;
  /* streams inflated per path (counted whether timing is on or not):
   * [0] sync-point two-phase, [1] general speculative (streams without sync
   * points), [2] one wave per stream */
  uint64_t inflate_paths[3];
  uint64_t general_passes; /* decode passes of the general path (1 = no redo) */
  /* deflate blocks whose bytes cannot beat a stored block (order-0 entropy
   * and no repeats): stored without a match search (counted whether timing
   * is on or not) */
  uint64_t blocks_unsearched;
} zt_kernel_times;
int zt_timing_enable(int on); /* resets the counters */
int zt_timing_read(zt_kernel_times *out);
/* Device scratch and pinned host staging the calling thread's device context
 * holds (grow-only caches reused by later calls), and a call that gives them
 * back (engine extension: the reference allocates per call, nothing is
 * cached). */
int zt_scratch_bytes(size_t *device_bytes, size_t *pinned_bytes);
int zt_release_scratch(void);

#ifdef __cplusplus
}
#endif
#endif
