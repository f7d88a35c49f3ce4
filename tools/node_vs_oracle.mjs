// Times the REFERENCE's RawDeflate + RawInflate (compiled js/, copied to a
// throw-away /tmp directory as tools/gen_golden.mjs does) on the sample files
// given on the command line; prints one JSON line.  Used once by
// tools/node_vs_oracle.py to record the speed ratio of the C restatement
// (oracle/, bench.py's cpu_baseline) to the reference itself (BASELINE.md).
import fs from 'fs';
import os from 'os';
import path from 'path';
import url from 'url';

const REF = '/root/reference/js';
if (!fs.existsSync(REF)) { console.error('reference absent'); process.exit(2); }
const shim = fs.mkdtempSync(path.join(os.tmpdir(), 'zref-'));
for (const f of fs.readdirSync(REF)) if (f.endsWith('.js')) fs.copyFileSync(path.join(REF, f), path.join(shim, f));
fs.writeFileSync(path.join(shim, 'package.json'), '{"type":"module"}');
fs.symlinkSync('Bitstream.js', path.join(shim, 'BitStream.js'));
(async () => {
  const { RawDeflate } = await import(url.pathToFileURL(path.join(shim, 'RawDeflate.js')).href);
  const { RawInflate } = await import(url.pathToFileURL(path.join(shim, 'RawInflate.js')).href);
  let bytes = 0, tdef = 0, tinf = 0, comp = 0;
  for (const f of process.argv.slice(2)) {
    const d = new Uint8Array(fs.readFileSync(f));
    let t0 = process.hrtime.bigint();
    const s = new RawDeflate(d).compress();
    let t1 = process.hrtime.bigint();
    const back = new RawInflate(s).decompress();
    let t2 = process.hrtime.bigint();
    if (back.length !== d.length) throw new Error('round trip');
    bytes += d.length; comp += s.length;
    tdef += Number(t1 - t0) / 1e9; tinf += Number(t2 - t1) / 1e9;
  }
  console.log(JSON.stringify({ bytes, compressed: comp, deflate_s: tdef, inflate_s: tinf, node: process.version }));
})();
