// GZip with the reference's surface (src/GZip.ts:40-194): same options
// (filename, comment, hcrc, deflateOptions), fields (input, ip, output, op,
// crc32, flags, filename, comment, deflateOptions) and return value.  The
// member is built by libzt (zt_gzip_compress): one upload of the input feeds
// both the GPU deflate pipeline and the GPU CRC-32.
import native, { dflt, refError } from './native.js';
import { CompressionType } from './Constants.js';

export const GZipMagicNumber = [0x1f, 0x8b];
export const GZipFlagsMask = { FTEXT: 0x01, FHCRC: 0x02, FEXTRA: 0x04, FNAME: 0x08, FCOMMENT: 0x10 };
export const GZipOperatingSystem = {
    FAT: 0, AMIGA: 1, VMS: 2, UNIX: 3, VM_CMS: 4, ATARI_TOS: 5, HPFS: 6, MACINTOSH: 7, Z_SYSTEM: 8,
    CP_M: 9, TOPS_20: 10, NTFS: 11, QDOS: 12, ACORN_RISCOS: 13, UNKNOWN: 255,
};

// header string -> bytes as src/GZip.ts:133-150 writes them (charCode > 0xFF: two LE bytes)
export function headerBytes(s) {
    const out = [];
    for (let i = 0; i < s.length; ++i) {
        const c = s.charCodeAt(i);
        if (c > 0xFF) out.push(c & 0xFF, (c >>> 8) & 0xFF);
        else out.push(c);
    }
    return Uint8Array.from(out);
}

export class GZip {
    constructor(input, opts = {}) {
        this.input = input;
        this.ip = 0;
        this.output = null;
        this.op = 0;
        this.crc32 = null;
        this.flags = {};
        this.filename = '';
        this.comment = '';
        if (opts.filename) {
            this.filename = opts.filename;
            this.flags.fname = true;
        }
        if (opts.comment) {
            this.comment = opts.comment;
            this.flags.fcomment = true;
        }
        if (opts.hcrc) this.flags.fhcrc = true;
        this.deflateOptions = dflt(opts.deflateOptions, {});
        // engine extension: a fixed MTIME (the reference always writes the current time)
        this.mtime = opts.mtime;
    }

    compress() {
        const d = this.input instanceof Uint8Array ? this.input : new Uint8Array(this.input);
        const o = this.deflateOptions;
        const ct = dflt(o.compressionType, CompressionType.DYNAMIC);
        const mtime = dflt(this.mtime, Math.floor(Date.now() / 1000));
        let r;
        try {
            r = native.gzipCompress(d, ct, dflt(o.lazy, 0), dflt(o.level, 6),
                this.flags.fname ? headerBytes(this.filename) : null,
                this.flags.fcomment ? headerBytes(this.comment) : null, !!this.flags.fhcrc, mtime >>> 0);
        } catch (e) {
            if (e.ztStatus === -1) throw 'invalid compression type';  // src/RawDeflate.ts:110 throws a string
            throw refError(e);
        }
        this.crc32 = r.crc32;
        this.output = r.output;
        this.op = r.output.length - 8;  // RawDeflate.op: end of the DEFLATE stream (src/GZip.ts:166)
        return r.output;
    }
}
