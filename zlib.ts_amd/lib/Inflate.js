// zlib Inflate with the reference's surface (src/Inflate.ts:15-93): the
// constructor validates CMF/FLG and throws the reference's errors;
// decompress() inflates on the GPU and, with `verify`, checks the Adler-32
// (libzt zt_zlib_decompress).  `ip` is the reference's: past the stream.
import native, { dflt, refError } from './native.js';

export class Inflate {
    constructor(input, opts = {}) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.index = dflt(opts.index, 0);
        this.ip = this.index;
        this.verify = dflt(opts.verify, false);
        this.adler32 = undefined;
        const cmf = this.input[this.ip++];
        const flg = this.input[this.ip++];
        if ((cmf & 0x0f) != 8) throw new Error('unsupported compression method');
        if (((cmf << 8) + flg) % 31 !== 0) throw new Error('invalid fcheck flag:' + ((cmf << 8) + flg) % 31);
        if (flg & 0x20) throw new Error('fdict flag is not supported');
    }

    decompress() {
        let r;
        try {
            r = native.zlibDecompress(this.input, this.index, this.verify);
        } catch (e) {
            throw refError(e);
        }
        this.ip = r.ip;
        if (this.verify) this.adler32 = r.adler32;
        return r.output;
    }
}
