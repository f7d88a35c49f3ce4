// RawInflateStream with the reference's surface (src/RawInflateStream.ts:
// 17-120): new RawInflateStream(input, ip, bufferSize), decompress(newInput,
// ip) decodes what the input holds so far and returns the bytes this call
// produced; `ip` advances over the input used.  Decoding runs on the GPU
// (zt_inflate_raw_resume): each call decodes every block that lies completely
// in the input (the reference stops mid-block, at a symbol; the concatenated
// output is the same), with the last 32 KiB of output as match history.
// Unlike the reference (src/RawInflateStream.ts:256-258), stored blocks with
// a correct NLEN are accepted.
import native, { dflt, refError } from './native.js';
import { DefaultInflateBufferSize } from './Constants.js';

const WINDOW = 32768;

export class RawInflateStream {
    constructor(input, ip = 0, opt_buffersize = DefaultInflateBufferSize) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.ip = ip;
        this.bufferSize = opt_buffersize;
        this.bitpos = 0;      // bits of input[ip] already used
        this.window = new Uint8Array(0);
        this.bfinal = false;
        this.totalpos = 0;    // bytes produced so far
        this.output = new Uint8Array(0);
    }

    decompress(newInput, ip) {
        return this._run(newInput, ip, 0);
    }

    // The input is complete (no more will come): decodes what is left and
    // throws the reference's message when the stream is corrupt near its end
    // or ends before its final block (decompress() would wait for more input).
    finish(newInput, ip) {
        const out = this._run(newInput, ip, 1);
        if (!this.bfinal) throw new Error('input buffer is broken');
        return out;
    }

    _run(newInput, ip, finalInput) {
        if (newInput) this.input = newInput instanceof Uint8Array ? newInput : new Uint8Array(newInput);
        this.ip = dflt(ip, this.ip);
        if (this.bfinal) return new Uint8Array(0);
        if (this.ip >= this.input.length && !finalInput) return new Uint8Array(0);
        let r;
        try {
            r = native.inflateResume(this.input, this.ip * 8 + this.bitpos, this.window, finalInput);
        } catch (e) {
            throw refError(e);
        }
        this.ip = Math.floor(r.endBits / 8);
        this.bitpos = r.endBits % 8;
        this.bfinal = r.finished;
        this.totalpos += r.output.length;
        // match history for the next call: the last 32 KiB of output
        if (r.output.length >= WINDOW) {
            this.window = r.output.slice(r.output.length - WINDOW);
        } else if (r.output.length) {
            const keep = Math.min(this.window.length, WINDOW - r.output.length);
            const w = new Uint8Array(keep + r.output.length);
            w.set(this.window.subarray(this.window.length - keep), 0);
            w.set(r.output, keep);
            this.window = w;
        }
        this.output = r.output;
        return r.output;
    }
}
