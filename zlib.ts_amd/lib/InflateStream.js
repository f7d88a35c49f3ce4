// InflateStream with the reference's surface (src/InflateStream.ts:7-89):
// zlib (RFC 1950) stream decoding over RawInflateStream.  decompress(chunk)
// appends the chunk, checks the 2-byte header once (the reference's errors),
// returns the bytes decoded by this call and, with `verify`, checks the
// Adler-32 trailer once the final block and its 4 bytes have arrived (the
// reference reads the trailer from the wrong buffer, src/InflateStream.ts:47).
import { RawInflateStream } from './RawInflateStream.js';
import { Adler32 } from './Adler32.js';

export class InflateStream {
    constructor(input, ip = 0) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input || []);
        this.ip = ip;
        this.header = false;
        this.rawinflate = null;
        this.output = new Uint8Array(0);
        this.verify = true;
        this.adler = 1;
        this.checked = false;
    }

    readHeader() {
        const cmf = this.input[this.ip], flg = this.input[this.ip + 1];
        if (cmf === undefined || flg === undefined) return false;
        if ((cmf & 0x0f) != 8) throw new Error('unsupported compression method');
        if (((cmf << 8) + flg) % 31 !== 0) throw new Error('invalid fcheck flag:' + ((cmf << 8) + flg) % 31);
        if (flg & 0x20) throw new Error('fdict flag is not supported');
        this.ip += 2;
        this.header = true;
        this.rawinflate = new RawInflateStream(this.input, this.ip);
        return true;
    }

    decompress(input) {
        if (input && input.length) {
            const tmp = new Uint8Array(this.input.length + input.length);
            tmp.set(this.input, 0);
            tmp.set(input, this.input.length);
            this.input = tmp;
        }
        if (!this.header && !this.readHeader()) return new Uint8Array(0);
        const raw = this.rawinflate;
        const buffer = raw.decompress(this.input, raw.ip);
        if (buffer.length) this.adler = Adler32.update(this.adler, buffer);
        this.output = buffer;
        if (raw.bfinal && this.verify && !this.checked) {
            const p = raw.ip + (raw.bitpos ? 1 : 0);  // the trailer starts at the next byte boundary
            if (p + 4 <= this.input.length) {
                const want = ((this.input[p] << 24) | (this.input[p + 1] << 16) | (this.input[p + 2] << 8) |
                              this.input[p + 3]) >>> 0;
                this.checked = true;
                if (want !== this.adler >>> 0) throw new Error('invalid adler-32 checksum');
            }
        }
        return buffer;
    }
}
