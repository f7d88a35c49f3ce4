// RawDeflate with the reference's surface (src/RawDeflate.ts:43-114): same
// constructor options, public fields and return value; the compression runs in
// libzt on the GPU (zt_deflate_raw).  `level` (1..9, default 6) is this
// build's extra option; the reference has none.
import native, { dflt } from './native.js';
import { CompressionType, DefaultDeflateBufferSize } from './Constants.js';

export { CompressionType };

export class RawDeflate {
    constructor(input, opts = {}) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.lazy = dflt(opts.lazy, 0);
        this.compressionType = dflt(opts.compressionType, CompressionType.DYNAMIC);
        this.level = dflt(opts.level, 6);
        if (opts.outputBuffer) {
            this.output = opts.outputBuffer instanceof Uint8Array ? opts.outputBuffer : new Uint8Array(opts.outputBuffer);
        } else {
            this.output = new Uint8Array(DefaultDeflateBufferSize);
        }
        this.op = dflt(opts.outputIndex, 0);
    }

    // Returns bytes [0, op): any caller prefix in outputBuffer[0..outputIndex)
    // followed by the raw DEFLATE stream (src/RawDeflate.ts:87-114).
    compress() {
        const ct = this.compressionType;
        if (ct !== CompressionType.NONE && ct !== CompressionType.FIXED && ct !== CompressionType.DYNAMIC) {
            throw 'invalid compression type';  // src/RawDeflate.ts:110 throws a string
        }
        if (ct === CompressionType.NONE && this.input.length === 0) {
            return this.output;  // the reference's NONE loop writes nothing and returns its buffer
        }
        let stream;
        try {
            stream = native.deflateRaw(this.input, ct, this.lazy, this.level);
        } catch (e) {
            if (e.ztStatus === -1) throw 'invalid compression type';
            throw e;
        }
        const start = this.op;
        if (start === 0) {  // no caller prefix: the library's buffer itself (no copy)
            this.output = stream;
            this.op = stream.length;
            return stream;
        }
        const out = new Uint8Array(start + stream.length);
        out.set(this.output.subarray(0, Math.min(start, this.output.length)));
        out.set(stream, start);
        this.output = out;
        this.op = out.length;
        return out;
    }
}
