// tools/gen_golden.mjs -- generate parity fixtures from the REFERENCE itself.
//
// Runs ExaGraphica/zlib.ts's compiled JS (/root/reference/js) under Node and
// records its outputs as data-only fixtures in tests/golden/.  The reference
// sources are copied to a throw-away directory under /tmp (never into this
// repository) with two shims: a package.json {"type":"module"} and a
// BitStream.js -> Bitstream.js symlink (js/RawDeflate.js:4 imports the
// differently-cased name).  Refuses to run when /root/reference is absent
// (e.g. on the GPU box): the committed fixtures are what travels.
//
//   node --max-old-space-size=16384 tools/gen_golden.mjs [outdir]
//
// (the 1 GiB checksum pins and the large inflate cases need the bigger heap:
// Node 12's default heap aborts with an out-of-memory error)
//
// Input generators are restated in tests/gen.py; each fixture records the
// generator spec so Python can rebuild large inputs instead of storing them.
import fs from 'fs';
import os from 'os';
import path from 'path';
import crypto from 'crypto';
import zlib from 'zlib';
import url from 'url';

const REF = '/root/reference/js';
if (!fs.existsSync(REF)) {
  console.error('gen_golden: /root/reference is not present; refusing to run');
  process.exit(2);
}
const outdir = process.argv[2] || path.join(path.dirname(url.fileURLToPath(import.meta.url)), '..', 'tests', 'golden');

// ---- shim ---------------------------------------------------------------
const shim = fs.mkdtempSync(path.join(os.tmpdir(), 'zref-'));
for (const f of fs.readdirSync(REF)) if (f.endsWith('.js')) fs.copyFileSync(path.join(REF, f), path.join(shim, f));
fs.writeFileSync(path.join(shim, 'package.json'), '{"type":"module"}');
fs.symlinkSync('Bitstream.js', path.join(shim, 'BitStream.js'));
const imp = (m) => import(url.pathToFileURL(path.join(shim, m)).href);

// ---- generators (restated in tests/gen.py) --------------------------------
function xorshift32(seed, n) {
  let x = (seed >>> 0) || 0x9E3779B9;
  const out = new Uint8Array(n);
  for (let i = 0; i < n; i++) {
    x ^= x << 13; x >>>= 0;
    x ^= x >>> 17;
    x ^= x << 5; x >>>= 0;
    out[i] = x & 0xFF;
  }
  return out;
}
const VOCAB = ['the', 'of', 'and', 'deflate', 'huffman', 'window', 'stream', 'block',
  'lz77', 'match', 'literal', 'inflate', 'gpu', 'wave', 'lane', 'chunk'];
function wordsalad(seed, n) {
  let x = (seed >>> 0) || 0x9E3779B9;
  const out = new Uint8Array(n);
  let i = 0;
  while (i < n) {
    x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0;
    const w = VOCAB[x & 15] + (((x >>> 4) & 15) === 0 ? '.\n' : ' ');
    for (let k = 0; k < w.length && i < n; k++) out[i++] = w.charCodeAt(k);
  }
  return out;
}
function structured(seed, n) {
  // little-endian int32 series with small deltas
  let x = (seed >>> 0) || 0x9E3779B9;
  const out = new Uint8Array(n);
  let v = 0;
  for (let i = 0; i < n; i += 4) {
    x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0;
    v = (v + ((x & 0xFF) - 128)) | 0;
    for (let k = 0; k < 4 && i + k < n; k++) out[i + k] = (v >>> (8 * k)) & 0xFF;
  }
  return out;
}
function gen(spec) {
  if (spec.hex !== undefined) return Uint8Array.from(Buffer.from(spec.hex, 'hex'));
  if (spec.ascii !== undefined) return Uint8Array.from(Buffer.from(spec.ascii, 'latin1'));
  const f = { xorshift32, wordsalad, structured }[spec.gen];
  if (spec.gen === 'fill') return new Uint8Array(spec.n).fill(spec.byte);
  if (spec.gen === 'concat') {
    const parts = spec.parts.map(gen);
    const out = new Uint8Array(parts.reduce((a, p) => a + p.length, 0));
    let o = 0;
    for (const p of parts) { out.set(p, o); o += p.length; }
    return out;
  }
  if (!f) throw new Error('bad spec ' + JSON.stringify(spec));
  return f(spec.seed, spec.n);
}

const hex = (u8) => Buffer.from(u8.buffer, u8.byteOffset, u8.length).toString('hex');
const sha = (u8) => crypto.createHash('sha256').update(Buffer.from(u8.buffer, u8.byteOffset, u8.length)).digest('hex');
const INLINE = 4096;
function blob(u8) { return u8.length <= INLINE ? { len: u8.length, hex: hex(u8) } : { len: u8.length, sha256: sha(u8) }; }

async function main() {
  const { RawDeflate } = await imp('RawDeflate.js');
  const { RawInflate } = await imp('RawInflate.js');
  const { CRC32 } = await imp('CRC32.js');
  const { Adler32 } = await imp('Adler32.js');
  fs.mkdirSync(outdir, { recursive: true });

  // ---------------- checksums (src/CRC32.ts, src/Adler32.ts) ---------------
  const ck = [];
  const ckInputs = [
    { ascii: '' }, { ascii: 'a' }, { ascii: 'abc' }, { ascii: '123456789' },
    { ascii: 'The quick brown fox jumps over the lazy dog' },
    { gen: 'xorshift32', seed: 1, n: 65536 },
    { gen: 'wordsalad', seed: 3, n: 100003 },
    { gen: 'structured', seed: 5, n: 5555 },
    { gen: 'fill', byte: 255, n: 70000 },
    { gen: 'xorshift32', seed: 11, n: 1 << 30 },
  ];
  for (let k = 0; k < 24; k++) ckInputs.push({ gen: 'xorshift32', seed: 1000 + k, n: (k * 7919) % 6007 });
  for (const spec of ckInputs) {
    const d = gen(spec);
    const rec = { input: spec.n > INLINE || (spec.gen && d.length > INLINE) ? spec : { hex: hex(d) },
      crc32: CRC32.create(d) >>> 0, adler32: Adler32.create(d) >>> 0 };
    if (d.length <= 100000) {
      // chained updates at a split point, as the containers do
      const cut = d.length >> 1;
      rec.crc32_chain = CRC32.update(d.subarray(cut), CRC32.create(d.subarray(0, cut))) >>> 0;
      rec.adler32_chain = Adler32.update(Adler32.create(d.subarray(0, cut)), d.subarray(cut)) >>> 0;
      // quirk: CRC32.create(data, pos) reads past the end (length defaults to data.length)
      if (d.length >= 3) rec.crc32_pos3 = CRC32.create(d, 3) >>> 0;
      // Adler32.update with len/pos
      if (d.length >= 10) rec.adler32_len_pos = Adler32.update(7, d, d.length - 5, 2) >>> 0;
    }
    ck.push(rec);
  }
  const singles = [];
  for (const [num, crc] of [[0, 0], [1, 0xFFFFFFFF], [0x41, 0x12345678], [255, 0xDEADBEEF], [300, 7]])
    singles.push({ num, crc, out: CRC32.single(num, crc) });
  // Adler32.create on a string (charCode & 0xFF, src/Util.ts:5-12)
  const strs = ['', 'Wikipedia', 'āĂzz'].map((s) => ({ str: s, adler32: Adler32.create(s) >>> 0 }));
  fs.writeFileSync(path.join(outdir, 'checksums.json'), JSON.stringify({ records: ck, singles, strings: strs }, null, 1));
  console.log('checksums:', ck.length);

  // ---------------- RawDeflate (src/RawDeflate.ts) -------------------------
  const df = [];
  const dfInputs = [
    { ascii: '' }, { ascii: 'A' }, { ascii: 'AB' }, { ascii: 'AAA' }, { ascii: 'AAAA' },
    { ascii: 'abcdeabcX' }, { ascii: 'hello hello hello' }, { ascii: 'abcabcabcabcabcabcX' },
    { ascii: 'Blah blah blah blah blah!' },
    { gen: 'fill', byte: 0, n: 1000 }, { gen: 'fill', byte: 97, n: 70000 },
    { gen: 'xorshift32', seed: 1, n: 65536 },
    { gen: 'xorshift32', seed: 2, n: 300 },
    { gen: 'wordsalad', seed: 1, n: 2000 }, { gen: 'wordsalad', seed: 2, n: 65536 },
    { gen: 'structured', seed: 1, n: 8192 },
    { gen: 'concat', parts: [{ gen: 'wordsalad', seed: 9, n: 20000 }, { gen: 'xorshift32', seed: 9, n: 20000 }, { gen: 'structured', seed: 9, n: 20000 }] },
  ];
  for (let k = 0; k < 16; k++) dfInputs.push({ gen: k & 1 ? 'wordsalad' : 'xorshift32', seed: 200 + k, n: 1 + ((k * 1237) % 3001) });
  const optsList = [{}, { compressionType: 1 }, { compressionType: 0 }, { lazy: 3 }, { lazy: 258 }, { compressionType: 1, lazy: 8 }];
  for (const spec of dfInputs) {
    const d = gen(spec);
    for (const opts of optsList) {
      if (d.length > 20000 && Object.keys(opts).length > 0 && !(opts.compressionType === 0)) continue;
      const rd = new RawDeflate(d, opts);
      let rec = { input: d.length > INLINE ? spec : { hex: hex(d) }, opts };
      try {
        const o = rd.compress();
        rec.out = blob(o); rec.op = rd.op;
        // round trip through the reference inflate (error recorded verbatim)
        try { rec.inflate_ok = sha(new RawInflate(o).decompress()) === sha(d); } catch (e) { rec.inflate_error = String(e.message || e); }
        rec.zlib_ok = (() => { try { return sha(new Uint8Array(zlib.inflateRawSync(Buffer.from(o)))) === sha(d); } catch (e) { return false; } })();
      } catch (e) { rec.error = String(e.message || e); }
      df.push(rec);
    }
  }
  // outputBuffer / outputIndex (callers: src/GZip.ts:159-160, src/Deflate.ts:41,84)
  for (const [prefix, idx, size] of [['78da', 2, 0x8000], ['1f8b0800', 4, 16], ['', 0, 8], ['aabbcc', 3, 3], ['aabbcc', 7, 4]]) {
    const d = gen({ ascii: 'hello hello hello hello world' });
    const ob = new Uint8Array(size);
    ob.set(Buffer.from(prefix, 'hex').subarray(0, size));
    const rd = new RawDeflate(d, { outputBuffer: ob, outputIndex: idx });
    const rec = { input: { hex: hex(d) }, opts: { outputBuffer: hex(ob), outputIndex: idx } };
    try { const o = rd.compress(); rec.out = blob(o); rec.op = rd.op; } catch (e) { rec.error = String(e.message || e); }
    df.push(rec);
  }
  // Uint16 heap truncation (src/Heap.ts:22): > 65535 occurrences of every literal
  {
    const spec = { gen: 'xorshift32', seed: 7, n: 18000000 };
    const d = gen(spec);
    const t0 = Date.now();
    const rd = new RawDeflate(d);
    const o = rd.compress();
    df.push({ input: spec, opts: {}, out: blob(o), op: rd.op, note: 'heap-uint16-truncation', ms: Date.now() - t0 });
  }
  for (const spec of [{ gen: 'wordsalad', seed: 4, n: 1 << 20 }, { gen: 'structured', seed: 4, n: 1 << 20 }]) {
    const d = gen(spec);
    const t0 = Date.now();
    const rd = new RawDeflate(d);
    const o = rd.compress();
    df.push({ input: spec, opts: {}, out: blob(o), op: rd.op, ms: Date.now() - t0 });
  }
  fs.writeFileSync(path.join(outdir, 'deflate.json'), JSON.stringify({ records: df }, null, 1));
  console.log('deflate:', df.length);

  // ---------------- RawInflate (src/RawInflate.ts) -------------------------
  const inf = [];
  fs.mkdirSync(path.join(outdir, 'streams'), { recursive: true });
  const record = (stream, opts, spec) => {
    const rec = { stream: blob(stream), opts, origin: spec };
    if (stream.length > INLINE) {
      // the stream itself is kept as a binary data file (tests/golden/streams/<sha16>.bin)
      rec.stream.file = 'streams/' + rec.stream.sha256.slice(0, 16) + '.bin';
      fs.writeFileSync(path.join(outdir, rec.stream.file), Buffer.from(stream.buffer, stream.byteOffset, stream.length));
    }
    try {
      const ri = new RawInflate(stream, opts);
      const o = ri.decompress();
      rec.out = blob(o); rec.ip = ri.ip;
    } catch (e) { rec.error = String(e.message || e); }
    inf.push(rec);
  };
  const infInputs = [
    { ascii: '' }, { ascii: 'x' }, { ascii: 'xy' }, { ascii: 'abcdeabcX' },
    { gen: 'wordsalad', seed: 21, n: 5000 }, { gen: 'xorshift32', seed: 21, n: 5000 },
    { gen: 'structured', seed: 21, n: 5000 }, { gen: 'fill', byte: 0, n: 40000 },
    { gen: 'concat', parts: [{ gen: 'wordsalad', seed: 22, n: 30000 }, { gen: 'xorshift32', seed: 22, n: 30000 }] },
  ];
  const C = zlib.constants;
  for (const spec of infInputs) {
    const d = gen(spec);
    for (const level of [0, 1, 6, 9]) {
      for (const strategy of [C.Z_DEFAULT_STRATEGY, C.Z_FIXED, C.Z_HUFFMAN_ONLY, C.Z_RLE]) {
        const s = new Uint8Array(zlib.deflateRawSync(Buffer.from(d), { level, strategy }));
        record(s, {}, { zlib: { input: spec, level, strategy } });
      }
    }
    // a stream produced by the reference itself
    const r = new RawDeflate(d).compress();
    record(r, {}, { refdeflate: { input: spec } });
  }
  // a few option variants: index (stream embedded after a prefix), BLOCK buffer mode, bufferSize
  for (const spec of [{ gen: 'wordsalad', seed: 31, n: 3000 }, { gen: 'wordsalad', seed: 32, n: 100000 }, { gen: 'xorshift32', seed: 33, n: 70000 }]) {
    const d = gen(spec);
    const s = new Uint8Array(zlib.deflateRawSync(Buffer.from(d), { level: 6 }));
    const pre = new Uint8Array(s.length + 7);
    pre.set([1, 2, 3, 4, 5, 6, 7]);
    pre.set(s, 7);
    record(pre, { index: 7 }, { zlib: { input: spec, level: 6 }, prefix: '01020304050607' });
    record(s, { bufferType: 0 }, { zlib: { input: spec, level: 6 } });
    record(s, { bufferSize: 1000 }, { zlib: { input: spec, level: 6 } });
    record(s, { bufferSize: 1 << 20, resize: true }, { zlib: { input: spec, level: 6 } });
  }
  // Z_SYNC_FLUSH-separated streams (byte-aligned empty stored blocks, as the GPU deflater emits)
  for (const spec of [{ gen: 'wordsalad', seed: 41, n: 50000 }, { gen: 'xorshift32', seed: 41, n: 50000 }]) {
    const d = gen(spec);
    const parts = [];
    for (let o = 0; o < d.length; o += 16384) {
      const last = o + 16384 >= d.length;
      parts.push(zlib.deflateRawSync(Buffer.from(d.subarray(Math.max(0, o - 0), o + 16384)), { level: 6, finishFlush: last ? C.Z_FINISH : C.Z_SYNC_FLUSH }));
    }
    // (independent members concatenated: only the last carries BFINAL)
    const s = new Uint8Array(Buffer.concat(parts));
    record(s, {}, { zlib_syncflush_16k: { input: spec, level: 6 } });
  }
  // malformed streams: reserved BTYPE, truncation, stored-length overrun
  for (const h of ['07', '06', '', '00', '0000', '000500faff', '010100feff41', '0300', 'ed']) record(Uint8Array.from(Buffer.from(h, 'hex')), {}, { hex: h });
  {
    const d = gen({ gen: 'wordsalad', seed: 51, n: 4000 });
    const s = new Uint8Array(zlib.deflateRawSync(Buffer.from(d), { level: 6 }));
    for (const cut of [1, 2, 3, 10, s.length >> 1, s.length - 2, s.length - 1]) record(s.subarray(0, cut), {}, { truncated: cut });
  }
  fs.writeFileSync(path.join(outdir, 'inflate.json'), JSON.stringify({ records: inf }, null, 1));
  console.log('inflate:', inf.length);
  fs.rmSync ? fs.rmSync(shim, { recursive: true, force: true }) : fs.rmdirSync(shim, { recursive: true });
}

main().catch((e) => { console.error(e); process.exit(1); });
