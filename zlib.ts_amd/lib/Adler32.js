// Adler32 with the reference's surface (src/Adler32.ts:7-58); the checksum
// runs in libzt on the GPU (zt_adler32_update).
import native, { dflt } from './native.js';

function stringToByteArray(s) {  // src/Util.ts:5-12: charCode & 0xFF
    const a = new Uint8Array(s.length);
    for (let i = 0; i < s.length; ++i) a[i] = s.charCodeAt(i) & 0xFF;
    return a;
}

export const Adler32 = {
    create(array) {
        if (typeof array === 'string') array = stringToByteArray(array);
        else if (!(array instanceof Uint8Array)) array = new Uint8Array(array);
        return this.update(1, array);
    },
    update(adler, array, len, pos = 0) {
        len = dflt(len, array.length);
        if (len <= 0) return ((((adler >> 16) & 0xFFFF) << 16) | (adler & 0xFFFF)) >>> 0;
        // reading past the end makes the reference's sums NaN, which >>> 0 turns into 0
        if (pos + len > array.length) return 0;
        return native.adler32Update(adler >>> 0, array.subarray(pos, pos + len));
    },
    OptimizationParameter: 1024,
};
