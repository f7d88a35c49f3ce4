// RawInflate with the reference's surface (src/RawInflate.ts:63-143): same
// options (index, bufferSize, bufferType, resize) and public fields (ip, op,
// buffer, output); decoding runs in libzt on the GPU (zt_inflate_raw).
// `refStrict: true` reproduces the reference's over-strict end-of-input check
// (src/RawInflate.ts:187) and its exact `ip` bookkeeping.
import native, { dflt } from './native.js';
import { BufferType, DefaultInflateBufferSize } from './Constants.js';

export { BufferType };

export class RawInflate {
    constructor(input, opts = {}) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.ip = dflt(opts.index, 0);
        this.bufferSize = dflt(opts.bufferSize, DefaultInflateBufferSize);
        this.bufferType = dflt(opts.bufferType, BufferType.ADAPTIVE);
        this.resize = dflt(opts.resize, false);
        this.refStrict = dflt(opts.refStrict, false);
        this.buffer = null;
        this.output = new Uint8Array(0);
        this.op = 0;
    }

    decompress() {
        if (this.bufferType !== BufferType.BLOCK && this.bufferType !== BufferType.ADAPTIVE) {
            throw new Error('invalid inflate mode');
        }
        let r;
        try {
            r = native.inflateRaw(this.input, this.ip, this.bufferType, this.bufferSize, this.refStrict);
        } catch (e) {
            // libzt's message is the reference's text ('input buffer is broken', ...)
            throw new Error(e.message);
        }
        this.ip = r.ip;
        this.output = r.output;
        this.op = r.output.length;
        this.buffer = r.output;
        return r.output;
    }
}
