// GUnzip with the reference's surface (src/GUnzip.ts:6-203): decompress()
// returns every member's data concatenated, getMembers() the parsed headers.
// Header parsing, the DEFLATE bodies (segment-parallel when they carry
// restart points) and the CRC-32 checks run in libzt (zt_gunzip).
import native, { refError } from './native.js';

const latin1 = (u8) => {
    let s = '';
    for (let i = 0; i < u8.length; ++i) s += String.fromCharCode(u8[i]);
    return s;
};

export class GUnzip {
    constructor(input) {
        this.input = input instanceof Uint8Array ? input : new Uint8Array(input);
        this.ip = 0;
        this.members = [];
        this.decompressed = false;
        this.crc32 = null;
    }

    getMembers() {
        if (!this.decompressed) this.decompress();
        return this.members.slice();
    }

    decompress() {
        let r;
        try {
            r = native.gunzip(this.input.subarray(this.ip));
        } catch (e) {
            throw refError(e);
        }
        const base = this.ip;
        for (const m of r.members) {
            const member = {
                id1: 0x1f, id2: 0x8b, cm: 8, flg: m.flg, mtime: new Date(m.mtime * 1000), xfl: m.xfl, os: m.os,
                data: r.output.subarray(m.dataOff, m.dataOff + m.dataLen),
            };
            if (m.flg & 0x04) member.xlen = m.xlen;
            if (m.flg & 0x08) member.name = latin1(this.input.subarray(base + m.nameOff, base + m.nameOff + m.nameLen));
            if (m.flg & 0x10) {
                member.comment = latin1(this.input.subarray(base + m.commentOff, base + m.commentOff + m.commentLen));
            }
            if (m.crc16 >= 0) member.crc16 = m.crc16;
            this.members.push(member);
            this.crc32 = m.crc32;
        }
        this.ip = this.input.length;
        this.decompressed = true;
        return r.output;
    }
}
