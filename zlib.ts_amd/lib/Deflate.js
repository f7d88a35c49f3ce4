// zlib Deflate with the reference's surface (src/Deflate.ts:16-99): CMF/FLG
// (FLEVEL = compressionType), raw DEFLATE and the big-endian Adler-32, built
// by libzt (zt_zlib_compress) from one device copy of the input.
import native, { dflt, refError } from './native.js';
import { CompressionType } from './Constants.js';

export class Deflate {
    constructor(input, opts = {}) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.output = new Uint8Array(0x8000);
        this.compressionType = dflt(opts.compressionType, CompressionType.DYNAMIC);
        this.lazy = dflt(opts.lazy, 0);
        this.level = dflt(opts.level, 6);
        this.adler32 = undefined;
    }

    static compress(input, opts) {
        return new Deflate(input, opts).compress();
    }

    compress() {
        let r;
        try {
            r = native.zlibCompress(this.input, this.compressionType, this.lazy, this.level);
        } catch (e) {
            if (e.ztStatus === -1) throw 'invalid compression type';
            throw refError(e);
        }
        this.adler32 = r.adler32;
        this.output = r.output;
        return r.output;
    }
}
