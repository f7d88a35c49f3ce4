/*
 * zt_oracle.c -- CPU restatement of ExaGraphica/zlib.ts (reference @ 2024-10-08).
 *
 * TEST INFRASTRUCTURE ONLY (see zt_oracle.h).  Not part of the product: the
 * engine in zlib.ts_amd/ never links this file.  It is the parity oracle for
 * the HIP kernels and the "port" CPU baseline in bench.py.
 *
 * Each function cites the reference file:line it restates.  JS semantics the
 * reference depends on are emulated explicitly:
 *   - typed-array writes past the end are dropped, reads past the end give
 *     `undefined` (ToNumber -> NaN -> 0 when stored into a Uint8Array);
 *   - Int32 arithmetic of the bitwise operators.
 */
#include "zt_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* CRC32  (src/CRC32.ts)                                                     */
/* ------------------------------------------------------------------------ */
static uint32_t crc_table[256];
static int crc_ready;

/* src/CRC32.ts:59-69 CRC32.init: reflected polynomial 0xEDB88320 */
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int j = 0; j < 8; ++j) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    crc_table[i] = c;
  }
  crc_ready = 1;
}

/* src/CRC32.ts:25-47 CRC32.update: XOR-in, byte table loop, XOR-out.  The
 * 8x unroll (lines 32-44) does not change the result. */
uint32_t zo_crc32_update(const uint8_t *data, size_t n, uint32_t crc) {
  if (!crc_ready) crc_init();
  crc ^= 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) crc = (crc >> 8) ^ crc_table[(crc ^ data[i]) & 0xFF];
  return crc ^ 0xFFFFFFFFu;
}

/* src/CRC32.ts:54-56 CRC32.single (no pre/post inversion) */
uint32_t zo_crc32_single(uint32_t num, uint32_t crc) {
  if (!crc_ready) crc_init();
  return crc_table[(num ^ crc) & 0xFF] ^ (crc >> 8);
}

/* ------------------------------------------------------------------------ */
/* Adler32  (src/Adler32.ts:28-48)                                          */
/* ------------------------------------------------------------------------ */
uint32_t zo_adler32_update(uint32_t adler, const uint8_t *a, size_t len) {
  uint64_t s1 = adler & 0xFFFF, s2 = (adler >> 16) & 0xFFFF;
  size_t pos = 0;
  while (len > 0) {
    size_t tlen = len > 1024 ? 1024 : len; /* OptimizationParameter, :57 */
    len -= tlen;
    do {
      s1 += a[pos++];
      s2 += s1;
    } while (--tlen);
    s1 %= 65521;
    s2 %= 65521;
  }
  return (uint32_t)((s2 << 16) | s1);
}

/* ------------------------------------------------------------------------ */
/* BitStream  (src/Bitstream.ts)                                             */
/* ------------------------------------------------------------------------ */
static uint8_t rev_table[256];
static int rev_ready;

/* src/Bitstream.ts:134-147 ReverseTable */
static void rev_init(void) {
  for (int i = 0; i < 256; ++i) {
    int r = i, s = 7, k = i;
    for (k >>= 1; k; k >>= 1) {
      r <<= 1;
      r |= k & 1;
      --s;
    }
    rev_table[i] = (uint8_t)((r << s) & 0xFF);
  }
  rev_ready = 1;
}

/* ReverseTable[x] with JS undefined -> 0 for x outside [0, 255] */
static inline int32_t rt(int64_t x) { return (x >= 0 && x < 256) ? rev_table[x] : 0; }

typedef struct {
  uint8_t *buf;
  size_t len;
  size_t index;
  int bitindex;
} bitstream_t;

/* src/Bitstream.ts:35-42 expandBuffer */
static void bs_expand(bitstream_t *s) {
  size_t nl = s->len << 1;
  uint8_t *nb = (uint8_t *)calloc(nl ? nl : 1, 1);
  if (s->len) memcpy(nb, s->buf, s->len);
  free(s->buf);
  s->buf = nb;
  s->len = nl;
}

/* src/Bitstream.ts:18-29 constructor (takes ownership of buf) */
static int bs_init(bitstream_t *s, uint8_t *buf, size_t len, size_t pos) {
  if (!rev_ready) rev_init();
  s->buf = buf;
  s->len = len;
  s->index = pos;
  s->bitindex = 0;
  if (s->len * 2 <= s->index) return ZO_ERR_INVALID_INDEX;
  if (s->len <= s->index) bs_expand(s);
  return ZO_OK;
}

/* src/Bitstream.ts:50-55 rev32 (Int32 result) */
static int32_t rev32(int32_t n) {
  uint32_t u = (uint32_t)n;
  uint32_t r = ((uint32_t)rt(u & 0xFF) << 24) | ((uint32_t)rt((u >> 8) & 0xFF) << 16) |
               ((uint32_t)rt((u >> 16) & 0xFF) << 8) | (uint32_t)rt((u >> 24) & 0xFF);
  return (int32_t)r;
}

#define UNDEF_BITS (-1) /* writeBits(x, undefined) */

/* src/Bitstream.ts:62-106 writeBits(number, b, reverse).  `b` may be
 * UNDEF_BITS (reference passes an out-of-range token entry): the loop then
 * runs zero times and only `buffer[index] = current` executes. */
static void bs_write(bitstream_t *s, int32_t number, int b, int reverse) {
  size_t index = s->index;
  int bitindex = s->bitindex;
  int32_t current = s->buf[index];
  if (b == UNDEF_BITS) {
    s->buf[index] = (uint8_t)current;
    return;
  }
  if (reverse && b > 1) {
    if (b > 8)
      number = rev32(number) >> ((32 - b) & 31);
    else
      number = rt(number) >> (8 - b);
  }
  if (b + bitindex < 8) {
    current = (int32_t)((uint32_t)current << b) | number;
    bitindex += b;
  } else {
    for (int i = 0; i < b; ++i) {
      current = (int32_t)((uint32_t)current << 1) | ((number >> ((b - i - 1) & 31)) & 1);
      if (++bitindex == 8) {
        bitindex = 0;
        s->buf[index++] = (uint8_t)rt(current);
        current = 0;
        if (index == s->len) bs_expand(s);
      }
    }
  }
  s->buf[index] = (uint8_t)current;
  s->index = index;
  s->bitindex = bitindex;
}

/* src/Bitstream.ts:112-130 finish: pad and return [0, index) */
static size_t bs_finish(bitstream_t *s) {
  if (s->bitindex > 0) {
    uint8_t v = (uint8_t)(s->buf[s->index] << (8 - s->bitindex));
    s->buf[s->index] = (uint8_t)rt(v);
    s->index++;
  }
  return s->index;
}

/* ------------------------------------------------------------------------ */
/* LZ77  (src/LZ77.ts)                                                       */
/* ------------------------------------------------------------------------ */
#define LZ_MIN 3
#define LZ_MAX 258
#define WINDOW 0x8000

/* src/LZ77.ts:20-53 getLengthCode -> [code, extra, bits] */
static int length_code(int length, int out[3]) {
  static const int lo[] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                           31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  static const int bits[] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                             2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  if (length < 3 || length > 258) return -1; /* throw 'invalid length: ' + n (:51) */
  int k = 28;
  if (length < 258) {
    k = 27;
    while (lo[k] > length) --k;
  }
  out[0] = 257 + k;
  out[1] = length - lo[k];
  out[2] = bits[k];
  return 0;
}

/* src/LZ77.ts:56-90 getDistanceCode -> [code, extra, bits] */
static int distance_code(int dist, int out[3]) {
  static const int lo[] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,
                           33,  49,  65,  97,  129, 193,  257,  385,  513,  769,
                           1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  static const int bits[] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                             6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  if (dist < 1 || dist > 32768) return -1; /* throw 'invalid distance' (:88) */
  int k = 29;
  while (lo[k] > dist) --k;
  out[0] = k;
  out[1] = dist - lo[k];
  out[2] = bits[k];
  return 0;
}

typedef struct {
  const uint8_t *in;
  size_t n;
  uint16_t *out; /* Uint16Array(2N), src/LZ77.ts:122 */
  size_t cap;
  size_t pos;
  long skip;
  int has_prev;
  int prev_len, prev_dist;
  int lazy;
  uint32_t fl[286];
  uint32_t fd[30];
  int err;
} lz_t;

/* src/LZ77.ts:131-133 writeNum: OOB typed-array writes are dropped */
static inline void lz_write_num(lz_t *z, int v) {
  if (z->pos < z->cap) z->out[z->pos] = (uint16_t)v;
  z->pos++;
}

/* src/LZ77.ts:135-146 writeMatch */
static void lz_write_match(lz_t *z, int len, int dist, int offset) {
  int lc[3], dc[3];
  if (length_code(len, lc) || distance_code(dist, dc)) {
    z->err = ZO_ERR_TYPE;
    return;
  }
  lz_write_num(z, lc[0]);
  lz_write_num(z, lc[1]);
  lz_write_num(z, lc[2]);
  lz_write_num(z, dc[0]);
  lz_write_num(z, dc[1]);
  lz_write_num(z, dc[2]);
  z->fl[lc[0]]++;
  z->fd[dc[0]]++;
  z->skip = len + offset - 1;
  z->has_prev = 0;
}

/* src/LZ77.ts:149-154 maxMatchTest */
static int lz_max_match_test(const lz_t *z, size_t m1, size_t m2, int len) {
  for (int j = len; j > LZ_MIN; j--)
    if (z->in[m1 + j - 1] != z->in[m2 + j - 1]) return 0;
  return 1;
}

/*
 * src/LZ77.ts:196-283 encode.  The reference keeps one JS array per exact
 * 24-bit key (:197,211-214) and evicts entries older than WindowSize from its
 * head (:223-225); walking an exact-key chain newest->oldest while
 * p - q <= 32768 visits exactly the same candidates in the same order.
 */
static int lz_encode(lz_t *z) {
  const uint8_t *in = z->in;
  size_t n = z->n;
  int32_t *head = (int32_t *)malloc(sizeof(int32_t) << 24);
  int32_t *prev = (int32_t *)malloc(sizeof(int32_t) * (n ? n : 1));
  if (!head || !prev) {
    free(head);
    free(prev);
    return ZO_ERR_TYPE;
  }
  memset(head, 0xFF, sizeof(int32_t) << 24);
  for (size_t p = 0; p < n; ++p) {
    uint32_t key = 0;
    for (int i = 0; i < LZ_MIN; i++) {
      if (p + i == n) break;
      key = (key << 8) | in[p + i];
    }
    key &= 0xFFFFFF;
    if ((z->skip--) > 0) { /* :217-220 */
      prev[p] = head[key];
      head[key] = (int32_t)p;
      continue;
    }
    if (p + LZ_MIN >= n) { /* :228-239 end-of-input literal flush */
      if (z->has_prev) lz_write_match(z, z->prev_len, z->prev_dist, -1);
      for (size_t i = p; i < n; i++) {
        lz_write_num(z, in[i]);
        z->fl[in[i]]++;
      }
      break;
    }
    int32_t q0 = head[key];
    int has_cand = (q0 >= 0 && (long)p - q0 <= WINDOW);
    if (has_cand) {
      /* :157-194 searchLongestMatch over the list newest -> oldest */
      long cur = q0;
      int match_max = 0;
      for (int32_t q = q0; q >= 0 && (long)p - q <= WINDOW; q = prev[q]) {
        int ml = LZ_MIN;
        if (match_max > LZ_MIN) {
          if (!lz_max_match_test(z, (size_t)q, p, match_max)) continue;
          ml = match_max;
        }
        while (ml < LZ_MAX && p + ml < n && in[q + ml] == in[p + ml]) ml++;
        if (ml > match_max) {
          cur = q;
          match_max = ml;
        }
        if (ml == LZ_MAX) break;
      }
      int lm_len = match_max, lm_dist = (int)((long)p - cur);
      if (z->has_prev) { /* :245-258 */
        if (z->prev_len < lm_len) {
          int tmp = in[p - 1];
          lz_write_num(z, tmp);
          z->fl[tmp]++;
          lz_write_match(z, lm_len, lm_dist, 0);
        } else {
          lz_write_match(z, z->prev_len, z->prev_dist, -1);
        }
      } else if (lm_len < z->lazy) { /* :259-260 */
        z->has_prev = 1;
        z->prev_len = lm_len;
        z->prev_dist = lm_dist;
      } else {
        lz_write_match(z, lm_len, lm_dist, 0);
      }
    } else if (z->has_prev) { /* :264-266 */
      lz_write_match(z, z->prev_len, z->prev_dist, -1);
    } else { /* :267-272 */
      lz_write_num(z, in[p]);
      z->fl[in[p]]++;
    }
    if (z->err) break;
    prev[p] = head[key]; /* :274 matchList.push(position) */
    head[key] = (int32_t)p;
  }
  /* :278-279 terminate */
  lz_write_num(z, 256);
  z->fl[256]++;
  free(head);
  free(prev);
  return z->err;
}

static int lz_run(const uint8_t *in, size_t n, int lazy, lz_t *z) {
  memset(z, 0, sizeof(*z));
  z->in = in;
  z->n = n;
  z->cap = 2 * n;
  z->out = (uint16_t *)malloc(sizeof(uint16_t) * (z->cap ? z->cap : 1));
  z->lazy = lazy;
  z->fl[256] = 1; /* :127 */
  int rc = lz_encode(z);
  if (z->pos > z->cap) z->pos = z->cap; /* :281 subarray(0, pos) clamps */
  return rc;
}

int zo_lz77_encode(const uint8_t *in, size_t n, int lazy, uint16_t **tokens, size_t *ntokens,
                   uint32_t freqs_litlen[286], uint32_t freqs_dist[30]) {
  lz_t z;
  int rc = lz_run(in, n, lazy, &z);
  *tokens = z.out;
  *ntokens = z.pos;
  memcpy(freqs_litlen, z.fl, sizeof(z.fl));
  memcpy(freqs_dist, z.fd, sizeof(z.fd));
  return rc;
}

/* ------------------------------------------------------------------------ */
/* Heap  (src/Heap.ts) -- values stored in a Uint16Array (:22)               */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint16_t buf[4 * 286]; /* new Heap(2*HUFMAX) -> Uint16Array(size*2) */
  int length;
  int nodes;
} heap_t;

/* src/Heap.ts:49-81 push */
static void heap_push(heap_t *h, int index, uint32_t value) {
  uint16_t *heap = h->buf;
  int current = h->length;
  heap[h->length++] = (uint16_t)value; /* Uint16 truncation */
  heap[h->length++] = (uint16_t)index;
  h->nodes++;
  while (current > 0) {
    int parent = ((current - 2) >> 2) << 1;
    if (heap[current] > heap[parent]) {
      uint16_t t = heap[current];
      heap[current] = heap[parent];
      heap[parent] = t;
      t = heap[current + 1];
      heap[current + 1] = heap[parent + 1];
      heap[parent + 1] = t;
      current = parent;
    } else {
      break;
    }
  }
}

/* src/Heap.ts:88-132 pop */
static void heap_pop(heap_t *h, int *index, uint32_t *value) {
  uint16_t *heap = h->buf;
  *value = heap[0];
  *index = heap[1];
  h->nodes--;
  h->length -= 2;
  heap[0] = heap[h->length];
  heap[1] = heap[h->length + 1];
  int parent = 0;
  for (;;) {
    int current = 2 * parent + 2;
    if (current >= h->length) break;
    if (current + 2 < h->length && heap[current + 2] > heap[current]) current += 2;
    if (heap[current] > heap[parent]) {
      uint16_t t = heap[parent];
      heap[parent] = heap[current];
      heap[current] = t;
      t = heap[parent + 1];
      heap[parent + 1] = heap[current + 1];
      heap[current + 1] = t;
    } else {
      break;
    }
    parent = current;
  }
}

/* ------------------------------------------------------------------------ */
/* reversePackageMerge  (src/RawDeflate.ts:484-571)                          */
/* value[][] entries are doubles with NaN = JS undefined; type[][] entries   */
/* use -1 for undefined.                                                     */
/* ------------------------------------------------------------------------ */
typedef struct {
  int limit, symbols;
  const double *freqs; /* sorted descending, length `symbols` */
  uint8_t *code_length;
  int mc[32];
  double *value[32];
  int *type[32];
  int cur[32];
  int err;
} pm_t;

static inline double pm_freq(const pm_t *s, int i) { return (i >= 0 && i < s->symbols) ? s->freqs[i] : NAN; }
static inline double pm_val(const pm_t *s, int j, int t) { return (t >= 0 && t < s->mc[j]) ? s->value[j][t] : NAN; }
static inline int pm_type(const pm_t *s, int j, int t) { return (t >= 0 && t < s->mc[j]) ? s->type[j][t] : -1; }

/* :496-507 takePackage */
static void pm_take(pm_t *s, int j) {
  if (j >= s->limit) { /* type[limit] is undefined -> TypeError */
    s->err = ZO_ERR_TYPE;
    return;
  }
  int x = pm_type(s, j, s->cur[j]);
  if (x == s->symbols) {
    pm_take(s, j + 1);
    pm_take(s, j + 1);
  } else if (x >= 0 && x < s->symbols) {
    s->code_length[x]--; /* Uint8Array wraps */
  }
  s->cur[j]++;
}

static int reverse_package_merge(const double *freqs, int symbols, int limit, uint8_t *code_length) {
  pm_t s;
  memset(&s, 0, sizeof(s));
  s.limit = limit;
  s.symbols = symbols;
  s.freqs = freqs;
  s.code_length = code_length;
  int flag[32] = {0};
  for (int i = 0; i < symbols; ++i) code_length[i] = (uint8_t)limit;
  /* minimumCost is a Uint16Array(limit) (:485) */
  uint16_t mc[32] = {0};
  mc[limit - 1] = (uint16_t)symbols;
  long excess = (1L << limit) - symbols;
  long half = 1L << (limit - 1);
  for (int j = 0; j < limit; ++j) {
    if (excess < half) {
      flag[j] = 0;
    } else {
      flag[j] = 1;
      excess -= half;
    }
    excess <<= 1;
    int idx = limit - 2 - j;
    if (idx >= 0) mc[idx] = (uint16_t)((mc[limit - 1 - j] >> 1) + symbols);
  }
  mc[0] = (uint16_t)flag[0];
  for (int j = 1; j < limit; ++j) {
    int cap = 2 * mc[j - 1] + flag[j];
    if (mc[j] > cap) mc[j] = (uint16_t)cap;
  }
  for (int j = 0; j < limit; ++j) {
    s.mc[j] = mc[j];
    s.value[j] = (double *)malloc(sizeof(double) * (mc[j] + 1));
    s.type[j] = (int *)malloc(sizeof(int) * (mc[j] + 1));
    for (int t = 0; t < mc[j]; ++t) {
      s.value[j][t] = NAN;
      s.type[j][t] = -1;
    }
  }
  for (int t = 0; t < mc[limit - 1]; ++t) {
    s.value[limit - 1][t] = pm_freq(&s, t);
    s.type[limit - 1][t] = t;
  }
  if (flag[limit - 1]) {
    if (symbols > 0) code_length[0]--;
    s.cur[limit - 1]++;
  }
  for (int j = limit - 2; j >= 0; j--) {
    int i = 0;
    int next = s.cur[j + 1];
    for (int t = 0; t < mc[j]; t++) {
      double weight = pm_val(&s, j + 1, next) + pm_val(&s, j + 1, next + 1);
      double fi = pm_freq(&s, i);
      if (weight > fi) { /* NaN compares false, as in JS */
        s.value[j][t] = weight;
        s.type[j][t] = symbols;
        next += 2;
      } else {
        s.value[j][t] = fi;
        s.type[j][t] = i;
        i++;
      }
    }
    s.cur[j] = 0;
    if (flag[j]) pm_take(&s, j);
    if (s.err) break;
  }
  for (int j = 0; j < limit; ++j) {
    free(s.value[j]);
    free(s.type[j]);
  }
  return s.err;
}

/* src/RawDeflate.ts:440-474 getLengths */
int zo_huffman_lengths(const uint32_t *freqs, size_t nsym, int limit, uint8_t *length) {
  heap_t h;
  memset(&h, 0, sizeof(h));
  memset(length, 0, nsym);
  for (size_t i = 0; i < nsym; ++i)
    if (freqs[i] > 0) heap_push(&h, (int)i, freqs[i]);
  int nnodes = h.nodes;
  if (nnodes == 1) {
    int idx;
    uint32_t v;
    heap_pop(&h, &idx, &v);
    if ((size_t)idx < nsym) length[idx] = 1;
    return ZO_OK;
  }
  int idxs[286];
  double values[286];
  for (int i = 0; i < nnodes; ++i) {
    uint32_t v;
    heap_pop(&h, &idxs[i], &v);
    values[i] = v;
  }
  uint8_t cl[286];
  int rc = reverse_package_merge(values, nnodes, limit, cl);
  if (rc) return rc;
  for (int i = 0; i < nnodes; ++i)
    if ((size_t)idxs[i] < nsym) length[idxs[i]] = cl[i];
  return ZO_OK;
}

/* src/RawDeflate.ts:580-611 getCodesFromLengths (returned bit-reversed) */
static void codes_from_lengths(const uint8_t *lengths, int n, uint16_t *codes) {
  int count[17] = {0};
  double start[17];
  for (int i = 0; i < n; i++)
    if (lengths[i] <= 16) count[lengths[i]]++;
  int code = 0;
  for (int i = 1; i <= 16; i++) {
    start[i] = code;
    code += count[i];
    code <<= 1;
  }
  for (int i = 0; i < n; i++) {
    int l = lengths[i];
    codes[i] = 0;
    if (l == 0) continue; /* startCode[0] is undefined; inner loop runs 0 times */
    uint32_t c = (uint32_t)start[l];
    start[l] += 1;
    uint16_t r = 0;
    for (int j = 0; j < l; j++) {
      r = (uint16_t)((r << 1) | (c & 1));
      c >>= 1;
    }
    codes[i] = r;
  }
}

/* src/RawInflate.ts:14 HuffmanOrder */
static const uint8_t huffman_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

/* src/RawDeflate.ts:341-431 getTreeSymbols (freqs is a Uint8Array: wraps) */
static int tree_symbols(int hlit, const uint8_t *ll, int hdist, const uint8_t *dl, uint32_t *result,
                        uint32_t *freqs32) {
  uint32_t src[316];
  uint8_t freqs[19] = {0};
  int l = hlit + hdist, j = 0, nres = 0;
  for (int i = 0; i < hlit; i++) src[j++] = ll[i];
  for (int i = 0; i < hdist; i++) src[j++] = dl[i];
  for (int i = 0; i < l; i += j) {
    for (j = 1; i + j < l && src[i + j] == src[i]; ++j) {
    }
    int run = j;
    if (src[i] == 0) {
      if (run < 3) {
        while (run-- > 0) {
          result[nres++] = 0;
          freqs[0]++;
        }
      } else {
        while (run > 0) {
          int rpt = run < 138 ? run : 138;
          if (rpt > run - 3 && rpt < run) rpt = run - 3;
          if (rpt <= 10) {
            result[nres++] = 17;
            result[nres++] = rpt - 3;
            freqs[17]++;
          } else {
            result[nres++] = 18;
            result[nres++] = rpt - 11;
            freqs[18]++;
          }
          run -= rpt;
        }
      }
    } else {
      result[nres++] = src[i];
      freqs[src[i]]++;
      run--;
      if (run < 3) {
        while (run-- > 0) {
          result[nres++] = src[i];
          freqs[src[i]]++;
        }
      } else {
        while (run > 0) {
          int rpt = run < 6 ? run : 6;
          if (rpt > run - 3 && rpt < run) rpt = run - 3;
          result[nres++] = 16;
          result[nres++] = rpt - 3;
          freqs[16]++;
          run -= rpt;
        }
      }
    }
  }
  for (int i = 0; i < 19; i++) freqs32[i] = freqs[i];
  return nres;
}

/* Token accessor with JS `undefined` (-1) past the end */
static inline int tok(const lz_t *z, size_t i) { return i < z->pos ? z->out[i] : -1; }

/* src/RawDeflate.ts:181-251 makeDynamicHuffmanBlock + :262-297 dynamicHuffman */
static int make_dynamic_block(bitstream_t *bs, const uint8_t *in, size_t n, int lazy, int final) {
  bs_write(bs, final ? 1 : 0, 1, 1);
  bs_write(bs, 2, 2, 1);
  lz_t z;
  int rc = lz_run(in, n, lazy, &z);
  if (rc) {
    free(z.out);
    return rc;
  }
  uint8_t ll[286], dl[30], tl[19];
  uint16_t lc[286], dc[30], tc[19];
  if ((rc = zo_huffman_lengths(z.fl, 286, 15, ll)) || (rc = zo_huffman_lengths(z.fd, 30, 7, dl))) {
    free(z.out);
    return rc;
  }
  codes_from_lengths(ll, 286, lc);
  codes_from_lengths(dl, 30, dc);
  int hlit, hdist, hclen;
  for (hlit = 286; hlit > 257 && ll[hlit - 1] == 0; hlit--) {
  }
  for (hdist = 30; hdist > 1 && dl[hdist - 1] == 0; hdist--) {
  }
  uint32_t tsym[316], tfreq[19];
  int ntsym = tree_symbols(hlit, ll, hdist, dl, tsym, tfreq);
  if ((rc = zo_huffman_lengths(tfreq, 19, 7, tl))) {
    free(z.out);
    return rc;
  }
  uint8_t trans[19];
  for (int i = 0; i < 19; i++) trans[i] = tl[huffman_order[i]];
  for (hclen = 19; hclen > 4 && trans[hclen - 1] == 0; hclen--) {
  }
  codes_from_lengths(tl, 19, tc);
  bs_write(bs, hlit - 257, 5, 1);
  bs_write(bs, hdist - 1, 5, 1);
  bs_write(bs, hclen - 4, 4, 1);
  for (int i = 0; i < hclen; i++) bs_write(bs, trans[i], 3, 1);
  for (int i = 0; i < ntsym; i++) {
    int code = (int)tsym[i];
    bs_write(bs, tc[code], tl[code], 1);
    if (code >= 16) {
      i++;
      int bitlen = code == 16 ? 2 : code == 17 ? 3 : 7;
      bs_write(bs, (int32_t)tsym[i], bitlen, 1);
    }
  }
  for (size_t idx = 0; idx < z.pos; ++idx) {
    int lit = z.out[idx];
    bs_write(bs, lc[lit], ll[lit], 1);
    if (lit > 256) {
      int v = tok(&z, ++idx), b = tok(&z, ++idx);
      bs_write(bs, v < 0 ? 0 : v, b, 1);
      int code = tok(&z, ++idx);
      if (code < 0)
        bs_write(bs, 0, UNDEF_BITS, 1);
      else
        bs_write(bs, dc[code], dl[code], 1);
      v = tok(&z, ++idx);
      b = tok(&z, ++idx);
      bs_write(bs, v < 0 ? 0 : v, b, 1);
    } else if (lit == 256) {
      break;
    }
  }
  free(z.out);
  return ZO_OK;
}

/* src/RawDeflate.ts:26-41 FixedHuffmanTable */
static void fixed_code(int lit, int *code, int *len) {
  if (lit <= 143) {
    *code = lit + 0x030;
    *len = 8;
  } else if (lit <= 255) {
    *code = lit - 144 + 0x190;
    *len = 9;
  } else if (lit <= 279) {
    *code = lit - 256;
    *len = 7;
  } else {
    *code = lit - 280 + 0x0C0;
    *len = 8;
  }
}

/* src/RawDeflate.ts:161-173 makeFixedHuffmanBlock + :305-330 fixedHuffman */
static int make_fixed_block(bitstream_t *bs, const uint8_t *in, size_t n, int lazy, int final) {
  bs_write(bs, final ? 1 : 0, 1, 1);
  bs_write(bs, 1, 2, 1);
  lz_t z;
  int rc = lz_run(in, n, lazy, &z);
  if (rc) {
    free(z.out);
    return rc;
  }
  for (size_t idx = 0; idx < z.pos; ++idx) {
    int lit = z.out[idx], code, len;
    fixed_code(lit, &code, &len);
    bs_write(bs, code, len, 0);
    if (lit > 0x100) {
      int v = tok(&z, ++idx), b = tok(&z, ++idx);
      bs_write(bs, v < 0 ? 0 : v, b, 1);
      v = tok(&z, ++idx);
      bs_write(bs, v < 0 ? 0 : v, 5, 0); /* dist code as 5 bits, MSB first (:320) */
      v = tok(&z, ++idx);
      b = tok(&z, ++idx);
      bs_write(bs, v < 0 ? 0 : v, b, 1);
    } else if (lit == 0x100) {
      break;
    }
  }
  free(z.out);
  return ZO_OK;
}

/* src/RawDeflate.ts:67-153  constructor + compress + makeNocompressBlock */
int zo_raw_deflate(const uint8_t *in, size_t n, int lazy, int ctype, const uint8_t *outbuf,
                   size_t outbuf_len, size_t out_index, uint8_t **out, size_t *out_len, size_t *op) {
  *out = NULL;
  *out_len = 0;
  size_t blen = outbuf ? outbuf_len : 0x8000; /* :73-78 */
  uint8_t *buf = (uint8_t *)calloc(blen ? blen : 1, 1);
  if (outbuf && blen) memcpy(buf, outbuf, blen);
  if (ctype == 0) { /* NONE, :93-100 */
    size_t cur_op = out_index;
    size_t cur_len = blen; /* underlying ArrayBuffer length */
    if (n == 0) {          /* no block written: returns the untouched buffer */
      *out = buf;
      *out_len = blen;
      *op = out_index;
      return ZO_OK;
    }
    for (size_t position = 0; position < n;) {
      size_t bl = n - position < 0xFFFF ? n - position : 0xFFFF;
      const uint8_t *blk = in + position;
      position += bl;
      int final = position == n;
      size_t len = cur_len;
      if (len == 0) {
        free(buf);
        return ZO_ERR_TYPE; /* `len <<= 1` never grows: the reference hangs */
      }
      while (len <= cur_op + bl + 5) len <<= 1;
      uint8_t *nb = (uint8_t *)calloc(len, 1); /* ByteStream.expandLength */
      memcpy(nb, buf, cur_len < len ? cur_len : len);
      free(buf);
      buf = nb;
      size_t p = cur_op;
      buf[p++] = (uint8_t)(final ? 1 : 0);
      buf[p++] = (uint8_t)(bl & 0xFF);
      buf[p++] = (uint8_t)((bl >> 8) & 0xFF);
      size_t nlen = bl ^ 0xFFFF;
      buf[p++] = (uint8_t)(nlen & 0xFF);
      buf[p++] = (uint8_t)((nlen >> 8) & 0xFF);
      memcpy(buf + p, blk, bl);
      p += bl;
      cur_op = p;
      cur_len = len;
    }
    *out = buf;
    *out_len = cur_op;
    *op = cur_op;
    return ZO_OK;
  }
  if (ctype != 1 && ctype != 2) {
    free(buf);
    return ZO_ERR_INVALID_COMPRESSION_TYPE;
  }
  bitstream_t bs;
  int rc = bs_init(&bs, buf, blen, out_index);
  if (rc) {
    free(bs.buf);
    return rc;
  }
  rc = ctype == 1 ? make_fixed_block(&bs, in, n, lazy, 1) : make_dynamic_block(&bs, in, n, lazy, 1);
  if (rc) {
    free(bs.buf);
    return rc;
  }
  size_t end = bs_finish(&bs);
  *out = bs.buf;
  *out_len = end;
  *op = end;
  return ZO_OK;
}

/* ------------------------------------------------------------------------ */
/* Huffman decode table  (src/Huffman.ts:8-68)                               */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t *table;
  int max_len;
  int min_len;
} htable_t;

static void build_huffman_table(const uint8_t *lengths, int n, htable_t *t) {
  int maxl = 0, minl = 1 << 30;
  for (int i = 0; i < n; ++i) {
    if (lengths[i] > maxl) maxl = lengths[i];
    if (lengths[i] < minl) minl = lengths[i];
  }
  size_t size = (size_t)1 << maxl;
  t->table = (uint32_t *)calloc(size, sizeof(uint32_t));
  t->max_len = maxl;
  t->min_len = minl;
  uint32_t code = 0;
  size_t skip = 2;
  for (int bl = 1; bl <= maxl;) {
    for (int i = 0; i < n; ++i) {
      if (lengths[i] == bl) {
        uint32_t rev = 0, rt_ = code;
        for (int j = 0; j < bl; ++j) {
          rev = (rev << 1) | (rt_ & 1);
          rt_ >>= 1;
        }
        uint32_t value = ((uint32_t)bl << 16) | (uint32_t)i;
        for (size_t j = rev; j < size; j += skip) t->table[j] = value;
        ++code;
      }
    }
    ++bl;
    code <<= 1;
    skip <<= 1;
  }
}

/* ------------------------------------------------------------------------ */
/* RawInflate  (src/RawInflate.ts)                                           */
/* ------------------------------------------------------------------------ */
static const uint16_t length_code_table[31] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  13,  15,
                                               17, 19, 23, 27, 31, 35, 43, 51,  59,  67,  83,
                                               99, 115, 131, 163, 195, 227, 258, 258, 258};
static const uint8_t length_extra_table[31] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                               3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0, 0, 0};
static const uint16_t dist_code_table[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,    25,
                                             33,   49,   65,   97,   129,  193,   257,   385,   513,   769,
                                             1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t dist_extra_table[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                             6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

typedef struct {
  const uint8_t *input;
  size_t ilen;
  size_t ip;
  uint32_t bitsbuf;
  int bitsbuflen;
  int bfinal;
  int mode; /* 0 BLOCK, 1 ADAPTIVE */
  uint8_t *output;
  size_t olen;
  size_t op;
  /* BLOCK mode */
  uint8_t **blocks;
  size_t *blens;
  size_t nblocks, cblocks;
  size_t totalpos;
  htable_t *cur_litlen;
  char *msg;
  size_t msg_cap;
  int err;
} inf_t;

static void inf_fail(inf_t *s, const char *m) {
  if (!s->err) {
    s->err = ZO_ERR_INFLATE;
    if (s->msg && s->msg_cap) snprintf(s->msg, s->msg_cap, "%s", m);
  }
}

/* src/RawInflate.ts:177-207 readBits, including the over-strict EOF check */
static uint32_t inf_read_bits(inf_t *s, int length) {
  if (s->err) return 0;
  long need = (long)(length - s->bitsbuflen + 7) >> 3; /* arithmetic >> */
  if ((long)s->ip + need >= (long)s->ilen) {
    inf_fail(s, "input buffer is broken");
    return 0;
  }
  while (s->bitsbuflen < length) {
    s->bitsbuf |= (uint32_t)s->input[s->ip++] << s->bitsbuflen;
    s->bitsbuflen += 8;
  }
  uint32_t octet = s->bitsbuf & ((1u << length) - 1);
  s->bitsbuf >>= length;
  s->bitsbuflen -= length;
  return octet;
}

/* src/RawInflate.ts:214-246 readCodeByTable */
static int inf_read_code(inf_t *s, const htable_t *t) {
  if (s->err) return 0;
  while (s->bitsbuflen < t->max_len) {
    if (s->ip >= s->ilen) break;
    s->bitsbuf |= (uint32_t)s->input[s->ip++] << s->bitsbuflen;
    s->bitsbuflen += 8;
  }
  uint32_t cwl = t->table[s->bitsbuf & ((1u << t->max_len) - 1)];
  int cl = (int)(cwl >> 16);
  if (cl > s->bitsbuflen) {
    char m[64];
    snprintf(m, sizeof m, "invalid code length: %d", cl);
    inf_fail(s, m);
    return 0;
  }
  s->bitsbuf >>= cl;
  s->bitsbuflen -= cl;
  return (int)(cwl & 0xFFFF);
}

/* src/RawInflate.ts:550-581 expandBufferAdaptive */
static void inf_expand_adaptive(inf_t *s, int add_ratio, int fix_ratio) {
  size_t ratio = (size_t)floor((double)s->ilen / (double)s->ip + 1);
  ratio = (fix_ratio ? (size_t)fix_ratio : ratio) + (size_t)add_ratio;
  size_t new_size;
  if (ratio < 2) {
    /* maxHuffCode = (len - ip) / minLen; Infinity when minLen == 0 */
    double min_len = s->cur_litlen ? s->cur_litlen->min_len : 0;
    double max_huff = (double)(s->ilen - s->ip) / min_len;
    double max_inflate = floor(max_huff * 129);
    new_size = max_inflate < (double)s->olen ? s->olen + (size_t)max_inflate : s->olen << 1;
  } else {
    new_size = s->olen * ratio;
  }
  uint8_t *nb = (uint8_t *)calloc(new_size ? new_size : 1, 1);
  memcpy(nb, s->output, s->olen < new_size ? s->olen : new_size);
  free(s->output);
  s->output = nb;
  s->olen = new_size;
}

/* src/RawInflate.ts:523-543 expandBufferBlock (copies the wrong range, :530) */
static void inf_expand_block(inf_t *s) {
  size_t blen = s->op - 32768;
  uint8_t *b = (uint8_t *)calloc(blen ? blen : 1, 1);
  /* buffer.set(output.subarray(MaxBackwardLength, buffer.length)) */
  if (blen > 32768) memcpy(b, s->output + 32768, blen - 32768);
  if (s->nblocks == s->cblocks) {
    s->cblocks = s->cblocks ? 2 * s->cblocks : 8;
    s->blocks = (uint8_t **)realloc(s->blocks, sizeof(uint8_t *) * s->cblocks);
    s->blens = (size_t *)realloc(s->blens, sizeof(size_t) * s->cblocks);
  }
  s->blocks[s->nblocks] = b;
  s->blens[s->nblocks++] = blen;
  s->totalpos += blen;
  memmove(s->output, s->output + (s->op - 32768), 32768);
  s->op = 32768;
}

/* Uint8Array element read with undefined -> 0 (distance before the start) */
static inline uint8_t inf_out_at(const inf_t *s, long i) {
  return (i >= 0 && (size_t)i < s->olen) ? s->output[i] : 0;
}

/* src/RawInflate.ts:407-459 (BLOCK) and :466-516 (ADAPTIVE) */
static void inf_decode_huffman(inf_t *s, htable_t *litlen, htable_t *dist) {
  s->cur_litlen = litlen;
  size_t olength = s->mode == 1 ? s->olen : s->olen - 258;
  int code;
  while (!s->err && (code = inf_read_code(s, litlen)) != 256) {
    if (s->err) return;
    if (code < 256) {
      if (s->op >= olength) {
        if (s->mode == 1) {
          inf_expand_adaptive(s, 0, 0);
          olength = s->olen;
        } else {
          inf_expand_block(s);
        }
      }
      if (s->op < s->olen) s->output[s->op] = (uint8_t)code;
      s->op++;
      continue;
    }
    int ti = code - 257;
    int len = ti < 31 ? length_code_table[ti] : 0;
    if (ti < 31 && length_extra_table[ti] > 0) len += (int)inf_read_bits(s, length_extra_table[ti]);
    int dcode = inf_read_code(s, dist);
    if (s->err) return;
    int dist_undef = dcode >= 30;
    long cdist = dist_undef ? 0 : dist_code_table[dcode];
    if (!dist_undef && dist_extra_table[dcode] > 0) cdist += inf_read_bits(s, dist_extra_table[dcode]);
    if (s->err) return;
    if (s->mode == 1) {
      if (s->op + (size_t)len > olength) {
        inf_expand_adaptive(s, 0, 0);
        olength = s->olen;
      }
    } else if (s->op >= olength) {
      inf_expand_block(s);
    }
    while (len--) {
      uint8_t v = dist_undef ? 0 : inf_out_at(s, (long)s->op - cdist);
      if (s->op < s->olen) s->output[s->op] = v;
      s->op++;
    }
  }
  if (s->err) return;
  while (s->bitsbuflen >= 8) { /* give back whole unread bytes */
    s->bitsbuflen -= 8;
    s->ip--;
  }
}

/* src/RawInflate.ts:251-318 parseUncompressedBlock */
static void inf_stored(inf_t *s) {
  s->bitsbuf = 0;
  s->bitsbuflen = 0;
  if (s->ip + 1 >= s->ilen) {
    inf_fail(s, "invalid uncompressed block header: LEN");
    return;
  }
  size_t len = s->input[s->ip] | ((size_t)s->input[s->ip + 1] << 8);
  s->ip += 2;
  if (s->ip + 1 >= s->ilen) {
    inf_fail(s, "invalid uncompressed block header: NLEN");
    return;
  }
  s->ip += 2; /* nlen: the `len === ~nlen` check (:277) can never fire */
  if (s->ip + len > s->ilen) {
    inf_fail(s, "input buffer is broken");
    return;
  }
  if (s->mode == 1) {
    while (s->op + len > s->olen) inf_expand_adaptive(s, 0, 2);
  } else {
    while (s->op + len > s->olen) {
      size_t pre = s->olen - s->op;
      len -= pre;
      memcpy(s->output + s->op, s->input + s->ip, pre);
      s->op += pre;
      s->ip += pre;
      inf_expand_block(s);
    }
  }
  memcpy(s->output + s->op, s->input + s->ip, len);
  s->op += len;
  s->ip += len;
}

static int fixed_tables_ready;
static htable_t fixed_litlen, fixed_dist;

/* src/RawInflate.ts:345-400 parseDynamicHuffmanBlock */
static void inf_dynamic(inf_t *s) {
  int hlit = (int)inf_read_bits(s, 5) + 257;
  int hdist = (int)inf_read_bits(s, 5) + 1;
  int hclen = (int)inf_read_bits(s, 4) + 4;
  if (s->err) return;
  uint8_t cls[19] = {0};
  for (int i = 0; i < hclen; ++i) cls[huffman_order[i]] = (uint8_t)inf_read_bits(s, 3);
  if (s->err) return;
  htable_t clt;
  build_huffman_table(cls, 19, &clt);
  int total = hlit + hdist;
  uint8_t lt[320];
  memset(lt, 0, sizeof lt);
  int prev = 0;
  for (int i = 0; i < total && !s->err;) {
    int code = inf_read_code(s, &clt);
    if (s->err) break;
    int repeat;
    switch (code) {
      case 16:
        repeat = 3 + (int)inf_read_bits(s, 2);
        while (repeat--) {
          if (i < total) lt[i] = (uint8_t)prev;
          i++;
        }
        break;
      case 17:
        repeat = 3 + (int)inf_read_bits(s, 3);
        while (repeat--) {
          if (i < total) lt[i] = 0;
          i++;
        }
        prev = 0;
        break;
      case 18:
        repeat = 11 + (int)inf_read_bits(s, 7);
        while (repeat--) {
          if (i < total) lt[i] = 0;
          i++;
        }
        prev = 0;
        break;
      default:
        lt[i++] = (uint8_t)code;
        prev = code;
        break;
    }
  }
  free(clt.table);
  if (s->err) return;
  htable_t llt, dt;
  build_huffman_table(lt, hlit, &llt);
  build_huffman_table(lt + hlit, hdist, &dt);
  inf_decode_huffman(s, &llt, &dt);
  /* keep llt alive only while decoding; cur_litlen is reset per block */
  s->cur_litlen = NULL;
  free(llt.table);
  free(dt.table);
}

static void inf_fixed(inf_t *s) {
  if (!fixed_tables_ready) {
    uint8_t l[288], d[30];
    for (int i = 0; i < 288; ++i) l[i] = i <= 143 ? 8 : i <= 255 ? 9 : i <= 279 ? 7 : 8;
    for (int i = 0; i < 30; ++i) d[i] = 5;
    build_huffman_table(l, 288, &fixed_litlen);
    build_huffman_table(d, 30, &fixed_dist);
    fixed_tables_ready = 1;
  }
  inf_decode_huffman(s, &fixed_litlen, &fixed_dist);
  s->cur_litlen = NULL;
}

/* src/RawInflate.ts:145-170 parseBlock */
static void inf_block(inf_t *s) {
  uint32_t header = inf_read_bits(s, 3);
  if (s->err) return;
  if (header & 1) s->bfinal = 1;
  header >>= 1;
  switch (header) {
    case 0:
      inf_stored(s);
      break;
    case 1:
      inf_fixed(s);
      break;
    case 2:
      inf_dynamic(s);
      break;
    default: {
      char m[48];
      snprintf(m, sizeof m, "unknown BTYPE: %u", header);
      inf_fail(s, m);
    }
  }
}

int zo_raw_inflate(const uint8_t *in, size_t n, size_t index, int buffer_type, size_t buffer_size,
                   uint8_t **out, size_t *out_len, size_t *ip, char *msg, size_t msg_cap) {
  inf_t s;
  memset(&s, 0, sizeof s);
  s.input = in;
  s.ilen = n;
  s.ip = index;
  s.mode = buffer_type == 0 ? 0 : 1;
  s.msg = msg;
  s.msg_cap = msg_cap;
  if (msg && msg_cap) msg[0] = 0;
  *out = NULL;
  *out_len = 0;
  if (s.mode == 0) { /* :114-116 */
    s.op = 32768;
    s.olen = 32768 + buffer_size + 258;
  } else {
    s.op = 0;
    s.olen = buffer_size;
  }
  s.output = (uint8_t *)calloc(s.olen ? s.olen : 1, 1);
  if (s.mode == 1 && s.olen == 0) { /* expansion can never grow: the reference hangs */
    free(s.output);
    return ZO_ERR_TYPE;
  }
  while (!s.bfinal && !s.err) inf_block(&s);
  if (s.err) {
    free(s.output);
    for (size_t i = 0; i < s.nblocks; ++i) free(s.blocks[i]);
    free(s.blocks);
    free(s.blens);
    return s.err;
  }
  if (s.mode == 1) { /* :629-643 concatBufferDynamic */
    size_t len = s.op < s.olen ? s.op : s.olen;
    *out = s.output;
    *out_len = len;
  } else { /* :587-623 concatBufferBlock */
    size_t limit = s.totalpos + (s.op - 32768);
    uint8_t *buf = (uint8_t *)calloc(limit ? limit : 1, 1);
    size_t pos = 0;
    for (size_t i = 0; i < s.nblocks; ++i) {
      memcpy(buf + pos, s.blocks[i], s.blens[i]);
      pos += s.blens[i];
      free(s.blocks[i]);
    }
    memcpy(buf + pos, s.output + 32768, s.op - 32768);
    free(s.output);
    free(s.blocks);
    free(s.blens);
    *out = buf;
    *out_len = limit;
  }
  *ip = s.ip;
  return ZO_OK;
}

void zo_free(void *p) { free(p); }

/* ------------------------------------------------------------------------ */
/* Synthetic input generators (test data); restated from    */
/* tools/gen_golden.mjs so fixtures can name large inputs by spec.          */
/* ------------------------------------------------------------------------ */
static inline uint32_t xs32(uint32_t x) {
  x ^= x << 13;
  x ^= x >> 17;
  x ^= x << 5;
  return x;
}

void zo_gen(int kind, uint32_t seed, uint8_t *out, size_t n) {
  static const char *vocab[16] = {"the",   "of",      "and",   "deflate", "huffman", "window",
                                  "stream", "block",  "lz77",  "match",   "literal", "inflate",
                                  "gpu",   "wave",    "lane",  "chunk"};
  uint32_t x = seed ? seed : 0x9E3779B9u;
  if (kind == 0) { /* xorshift32 */
    for (size_t i = 0; i < n; i++) {
      x = xs32(x);
      out[i] = (uint8_t)x;
    }
  } else if (kind == 1) { /* wordsalad */
    size_t i = 0;
    while (i < n) {
      x = xs32(x);
      const char *w = vocab[x & 15];
      for (; *w && i < n; w++) out[i++] = (uint8_t)*w;
      if (((x >> 4) & 15) == 0) {
        if (i < n) out[i++] = '.';
        if (i < n) out[i++] = '\n';
      } else if (i < n) {
        out[i++] = ' ';
      }
    }
  } else { /* structured: LE int32 series with small deltas */
    int32_t v = 0;
    for (size_t i = 0; i < n; i += 4) {
      x = xs32(x);
      v = (int32_t)((uint32_t)v + (uint32_t)((int32_t)(x & 0xFF) - 128));
      for (int k = 0; k < 4 && i + k < n; k++) out[i + k] = (uint8_t)((uint32_t)v >> (8 * k));
    }
  }
}
