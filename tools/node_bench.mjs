// The drop-in boundary timed from Node (BASELINE north_star: "host code stays
// TypeScript/Node calling HIP through a thin N-API C-ABI addon"): the
// reference's own call shapes, new RawDeflate(u8).compress() and
// new RawInflate(s).decompress() (src/RawDeflate.ts:87-114,
// src/RawInflate.ts:127-140), over the zlib.ts_amd facade and zt.node.
//   usage: node --expose-gc tools/node_bench.mjs [corpus_file] [reps]
// corpus_file: the bytes to round-trip (bench.py writes the 1 GiB bench
// corpus there); none: only the per-call latency below.  Prints one JSON line:
//   deflate / inflate / round trip GiB/s on the corpus (median of `reps`
//   timed calls, each after the previous results were collected -- so their
//   buffers are back in libzt's host output pool, the C-ABI bench's case),
//   and the C0-shaped per-call latency: 64 KiB of xorshift32 seed 1
//   (SURVEY 8(d)) deflated / inflated in a loop.
import fs from 'fs';
import { RawDeflate, RawInflate } from '../zlib.ts_amd/lib/index.js';

const gcRaw = typeof global.gc === 'function' ? global.gc : () => {};
// a collection, then one event-loop turn: N-API runs the external buffers'
// finalizers (zt_free) after the collection, not inside it
const gc = () => { gcRaw(); return new Promise((r) => setImmediate(r)); };
const now = () => Number(process.hrtime.bigint()) / 1e6;  // ms
const median = (a) => a.slice().sort((x, y) => x - y)[a.length >> 1];
const same = (a, b) => a.length === b.length &&
    Buffer.from(a.buffer, a.byteOffset, a.length).equals(Buffer.from(b.buffer, b.byteOffset, b.length));

function xorshift32(seed, n) {
    const out = new Uint8Array(n);
    let x = seed >>> 0;
    for (let i = 0; i < n; ++i) {
        x ^= x << 13; x >>>= 0;
        x ^= x >>> 17;
        x ^= x << 5; x >>>= 0;
        out[i] = x & 0xff;
    }
    return out;
}

const res = { node: process.version };
const file = process.argv[2];
const reps = Number(process.argv[3] || 3);
async function main() {
if (file) {
    const input = fs.readFileSync(file);  // a Buffer: a Uint8Array, as the reference takes
    const n = input.length;
    // warm-up (library scratch, staging, the host output pool)
    let s = new RawDeflate(input).compress();
    let back = new RawInflate(s).decompress();
    if (!same(back, input)) throw new Error('node bench: warm-up round trip mismatch');
    back = null;
    const td = [], ti = [];
    for (let r = 0; r < reps; ++r) {
        s = null;
        await gc();
        let t0 = now();
        s = new RawDeflate(input).compress();
        td.push(now() - t0);
        await gc();
        t0 = now();
        const inf = new RawInflate(s);
        back = inf.decompress();
        ti.push(now() - t0);
        if (inf.ip !== s.length || !same(back, input)) throw new Error('node bench: round trip mismatch');
        back = null;
    }
    const g = n / 2 ** 30;
    res.bytes = n;
    res.stream_bytes = s.length;
    res.deflate_ms = td.map((x) => +x.toFixed(2));
    res.inflate_ms = ti.map((x) => +x.toFixed(2));
    res.deflate_GiBps = +(g / (median(td) / 1e3)).toFixed(3);
    res.inflate_GiBps = +(g / (median(ti) / 1e3)).toFixed(3);
    res.roundtrip_GiBps = +(g / ((median(td) + median(ti)) / 1e3)).toFixed(3);
}
// C0 shape: 64 KiB random, one call at a time
const small = xorshift32(1, 65536);
let sm = new RawDeflate(small).compress();
for (let i = 0; i < 20; ++i) new RawInflate(new RawDeflate(small).compress()).decompress();
const calls = 200;
let t0 = now();
for (let i = 0; i < calls; ++i) sm = new RawDeflate(small).compress();
const usd = (now() - t0) * 1e3 / calls;
t0 = now();
let o;
for (let i = 0; i < calls; ++i) o = new RawInflate(sm).decompress();
const usi = (now() - t0) * 1e3 / calls;
if (!same(o, small)) throw new Error('node bench: 64 KiB round trip mismatch');
res.c0_64KiB = { stream_bytes: sm.length, deflate_us_per_call: +usd.toFixed(1), inflate_us_per_call: +usi.toFixed(1),
                 deflate_MiBps: +(65536 / 2 ** 20 / (usd / 1e6)).toFixed(1) };
console.log(JSON.stringify(res));
}
main().catch((e) => { console.error(e); process.exit(1); });
