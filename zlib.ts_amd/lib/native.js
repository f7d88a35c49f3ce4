// The N-API addon over libzt.so (include/zt.h).  There is no JS fallback: the
// hot path runs on the GPU, and loading fails loudly when the addon is absent.
import { createRequire } from 'module';
import { fileURLToPath } from 'url';
import path from 'path';

const here = path.dirname(fileURLToPath(import.meta.url));
const require = createRequire(import.meta.url);
let addon;
try {
    addon = require(path.join(here, '..', 'zt.node'));
} catch (e) {
    throw new Error('zlib.ts_amd: zt.node not built (make -C zlib.ts_amd zt.node): ' + e.message);
}
export default addon;

// libzt status codes (include/zt.h)
export const ZT = {
    INVALID_COMPRESSION_TYPE: -1,
    INPUT_BROKEN: -10,
};

// `a ?? b` (Node 12 has no nullish coalescing)
export function dflt(v, d) {
    return v === undefined || v === null ? d : v;
}

// libzt's message is the reference's text; keep the status code beside it
export function refError(e) {
    const err = new Error(e.message);
    if (e.ztStatus !== undefined) err.ztStatus = e.ztStatus;
    return err;
}
