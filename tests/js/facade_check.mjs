// Runs the JS facade (zlib.ts_amd/lib) over cases prepared by
// tests/test_js_facade.py and prints one JSON result per case.
import fs from 'fs';
import { RawDeflate, RawInflate, RawInflateStream, InflateStream, CRC32, Adler32, GZip, GUnzip, Deflate, Inflate, Zip, Unzip, deviceCount } from '../../zlib.ts_amd/lib/index.js';

const hex = (s) => Uint8Array.from(Buffer.from(s, 'hex'));
const tohex = (a) => Buffer.from(a.buffer, a.byteOffset, a.length).toString('hex');
const cases = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const out = [];
for (const c of cases) {
    const r = { id: c.id };
    try {
        if (c.op === 'devices') {
            r.value = deviceCount();
        } else if (c.op === 'crc32') {
            r.value = c.crc === undefined ? CRC32.create(hex(c.in), c.pos, c.length) : CRC32.update(hex(c.in), c.crc, c.pos, c.length);
        } else if (c.op === 'adler32') {
            r.value = c.str !== undefined ? Adler32.create(c.str) : Adler32.update(c.adler === undefined ? 1 : c.adler, hex(c.in), c.len, c.pos);
        } else if (c.op === 'inflate') {
            const inf = new RawInflate(hex(c.in), { index: c.index || 0, refStrict: !!c.strict, bufferType: c.bufferType === undefined ? 1 : c.bufferType });
            const o = inf.decompress();
            r.out = tohex(o);
            r.ip = inf.ip;
        } else if (c.op === 'deflate') {
            const opts = Object.assign({}, c.opts || {});
            if (c.prefix !== undefined) {
                opts.outputBuffer = hex(c.prefix);
                opts.outputIndex = c.prefix.length / 2;
            }
            const d = new RawDeflate(hex(c.in), opts);
            const s = d.compress();
            r.out = tohex(s);
            r.op = d.op;
            const body = s.subarray(opts.outputIndex || 0);
            const back = new RawInflate(body, { refStrict: true }).decompress();
            r.back = tohex(back);
        } else if (c.op === 'gzip') {
            const g = new GZip(hex(c.in), c.opts || {});
            r.out = tohex(g.compress());
            r.crc32 = g.crc32;
        } else if (c.op === 'gunzip') {
            const g = new GUnzip(hex(c.in));
            r.out = tohex(g.decompress());
            r.crc32 = g.crc32;
            r.members = g.getMembers().map((m) => ({
                flg: m.flg, xfl: m.xfl, os: m.os, mtime: Math.round(m.mtime.getTime() / 1000),
                name: m.name === undefined ? null : m.name, comment: m.comment === undefined ? null : m.comment,
                data: tohex(m.data),
            }));
        } else if (c.op === 'zlib') {
            const z = new Deflate(hex(c.in), c.opts || {});
            r.out = tohex(z.compress());
            r.adler32 = z.adler32;
        } else if (c.op === 'zinflate') {
            const z = new Inflate(hex(c.in), c.opts || {});
            r.out = tohex(z.decompress());
            r.ip = z.ip;
        } else if (c.op === 'zip') {
            // c.files: [{fn, in (hex), opts}], c.date: local-time components
            const z = new Zip(c.comment || []);
            for (const f of c.files) z.addFile(hex(f.in), f.fn, Object.assign({}, f.opts, { date: new Date(...c.date) }));
            r.out = tohex(z.compress());
        } else if (c.op === 'rstream') {
            // the stream arrives in pieces c.cuts (byte ends); every call is
            // given the whole input received so far, as the reference's callers do
            const all = hex(c.in);
            const st = new RawInflateStream(all.subarray(0, 0), 0);
            const parts = [];
            for (const end of c.cuts) parts.push(st.decompress(all.subarray(0, end)));
            r.out = parts.map(tohex).join('');
            r.calls = parts.map((x) => x.length);
            r.ip = st.ip;
            r.bitpos = st.bitpos;
            r.bfinal = st.bfinal;
        } else if (c.op === 'zstream') {
            // zlib stream in chunks appended by InflateStream.decompress(chunk)
            const all = hex(c.in);
            const st = new InflateStream(all.subarray(0, 0));
            const parts = [];
            let prev = 0;
            for (const end of c.cuts) {
                parts.push(st.decompress(all.subarray(prev, end)));
                prev = end;
            }
            r.out = parts.map(tohex).join('');
            r.checked = st.checked;
        } else if (c.op === 'unzip') {
            const u = new Unzip(hex(c.in), { verify: !!c.verify });
            r.names = u.getFilenames();
            r.files = r.names.map((nm) => {
                try {
                    return { name: nm, out: tohex(u.decompress(nm)) };
                } catch (e) {
                    return { name: nm, error: { message: e.message } };
                }
            });
        }
    } catch (e) {
        r.error = typeof e === 'string' ? { string: e } : { message: e.message, status: e.ztStatus };
    }
    out.push(r);
}
console.log(JSON.stringify(out));
