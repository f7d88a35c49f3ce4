// Unzip with the reference's surface (src/Unzip.ts:196-342): getFilenames(),
// decompress(filename), getFileData(index), parseFileHeader(), verify.  The
// first call decodes the whole archive in libzt (zt_unzip): the central
// directory and local headers are parsed with the reference's checks and
// messages and every DEFLATE member is inflated in one GPU batch; each
// getFileData(i) then returns entry i or throws its error as the reference
// would.  ZipCrypto is not supported.
import native, { refError } from './native.js';

function readString(input, off, len) {
    let s = '';
    for (let i = 0; i < len; ++i) s += String.fromCharCode(input[off + i]);
    return s;
}

export class Unzip {
    constructor(input, opts = {}) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.ip = 0;
        this.EOCD = null;
        this.verify = !!opts.verify;
        if (opts.password) this.password = opts.password;
        this.decoded = null;
    }

    decode() {
        if (this.decoded) return this.decoded;
        let r;
        try {
            r = native.unzip(this.input, this.verify);
        } catch (e) {
            throw refError(e);
        }
        this.decoded = r;
        return r;
    }

    parseFileHeader() {
        if (this.fileHeaderList) return;
        const r = this.decode();
        const list = [];
        const table = {};
        r.entries.forEach((e, i) => {
            const fh = Object.assign({}, e);
            fh.filename = readString(this.input, e.nameOff, e.nameLen);
            fh.fileNameLength = e.nameLen;
            fh.comment = this.input.subarray(e.commentOff, e.commentOff + e.commentLen);
            fh.fileCommentLength = e.commentLen;
            list[i] = fh;
            table[fh.filename] = i;
        });
        this.fileHeaderList = list;
        this.filenameToIndex = table;
    }

    getFileData(index) {
        this.parseFileHeader();
        const e = this.fileHeaderList[index];
        if (e === undefined) throw new Error('wrong index');
        if (e.status !== 0) throw new Error(e.message);
        return this.decoded.output.subarray(e.dataOff, e.dataOff + e.dataLen);
    }

    getFilenames() {
        this.parseFileHeader();
        return this.fileHeaderList.map((e) => e.filename);
    }

    decompress(filename) {
        this.parseFileHeader();
        const index = this.filenameToIndex[filename];
        if (index === undefined) throw new Error(filename + ' not found');
        return this.getFileData(index);
    }

    setPassword(password) {
        this.password = password;
    }
}
