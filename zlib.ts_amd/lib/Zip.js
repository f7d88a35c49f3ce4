// Zip with the reference's surface (src/Zip.ts:62-384): addFile(input,
// filename, opts), setPassword, compress(), the enums and the signatures.
// The archive is built by libzt (zt_zip_compress): every DEFLATE member of the
// archive is compressed in one GPU batch pipeline and every CRC-32 comes from
// the batched GPU checksum kernel; the layout is the reference's, byte for
// byte.  ZipCrypto is not supported (a password throws).
import native, { dflt, refError } from './native.js';
import { CompressionType } from './Constants.js';

export const ZipCompressionMethod = { STORE: 0, DEFLATE: 8 };
export const ZipOperatingSystem = { MSDOS: 0, UNIX: 3, MACINTOSH: 7 };
export const ZipFlags = { ENCRYPT: 0x0001, DESCRIPTOR: 0x0008, UTF8: 0x0800 };
export const FileHeaderSignature = new Uint8Array([0x50, 0x4b, 0x01, 0x02]);
export const LocalFileHeaderSignature = new Uint8Array([0x50, 0x4b, 0x03, 0x04]);
export const CentralDirectorySignature = new Uint8Array([0x50, 0x4b, 0x05, 0x06]);

// src/Util.ts stringToByteArray: one byte per UTF-16 unit (charCode & 0xFF)
export function stringToByteArray(str) {
    const tmp = new Uint8Array(str.length);
    for (let i = 0; i < tmp.length; i++) tmp[i] = str.charCodeAt(i) & 0xFF;
    return tmp;
}

// the DOS time / date bytes of src/Zip.ts:130-139
export function dosTime(date) {
    return new Uint8Array([
        ((date.getMinutes() & 0x7) << 5) | (date.getSeconds() >>> 1),
        (date.getHours() << 3) | (date.getMinutes() >> 3),
        ((date.getMonth() + 1 & 0x7) << 5) | (date.getDate()),
        ((date.getFullYear() - 1980 & 0x7f) << 1) | (date.getMonth() + 1 >> 3),
    ]);
}

export class Zip {
    constructor(comment = []) {
        this.files = [];
        this.comment = comment instanceof Uint8Array ? comment : new Uint8Array(comment);
        this.password = null;
    }

    // src/Zip.ts:80-108 (the engine compresses every member at compress(), in one batch)
    addFile(input, filename = '', opts = {}) {
        const buffer = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.files.push({
            filename,
            buffer,
            compressionMethod: dflt(opts.compressionMethod, ZipCompressionMethod.DEFLATE),
            option: opts,
            compressed: false,
            encrypted: false,
            size: buffer.length,
            crc32: 0,
        });
    }

    setPassword(password) {
        this.password = password;
    }

    compress() {
        const files = this.files.map((f) => {
            if (f.option.password !== undefined || this.password !== null) {
                throw new Error('zlib.ts_amd: ZipCrypto is not supported');
            }
            const date = f.option.date !== undefined && f.option.date !== null ? f.option.date : new Date();
            f.option.mtime = dosTime(date);
            const d = dflt(f.option.deflateOptions, {});
            return {
                data: f.buffer,
                name: stringToByteArray(f.filename),
                comment: f.option.comment ? stringToByteArray(f.option.comment) : null,
                method: f.compressionMethod,
                os: dflt(f.option.os, ZipOperatingSystem.MSDOS),
                mtime: f.option.mtime,
                compressionType: dflt(d.compressionType, CompressionType.DYNAMIC),
                lazy: dflt(d.lazy, 0),
                level: dflt(d.level, 6),
            };
        });
        try {
            return native.zipCompress(files, this.comment);
        } catch (e) {
            throw refError(e);
        }
    }
}
