// CRC32 with the reference's surface (src/CRC32.ts:5-72); the checksum runs in
// libzt on the GPU (zt_crc32_update).
import native, { dflt } from './native.js';

function bytes(data) {
    return data instanceof Uint8Array ? data : new Uint8Array(data);
}

const Table = new Uint32Array(256);
for (let i = 0; i < 256; ++i) {
    let c = i;
    for (let j = 0; j < 8; ++j) c = (c & 1) ? (0xEDB88320 ^ (c >>> 1)) : (c >>> 1);
    Table[i] = c >>> 0;
}

export const CRC32 = {
    create(data, pos, length) {
        return this.update(data, 0, pos, length);
    },
    // `length` defaults to data.length even when pos > 0 (src/CRC32.ts:27):
    // bytes past the end read as undefined, which the reference's table
    // lookup treats as 0 -- reproduced by zero padding.
    update(data, crc, pos = 0, length) {
        const d = bytes(data);
        const il = dflt(length, d.length);
        let view;
        if (pos + il <= d.length) {
            view = d.subarray(pos, pos + il);
        } else {
            view = new Uint8Array(il);
            if (pos < d.length) view.set(d.subarray(pos));
        }
        return native.crc32Update(view, crc >>> 0);
    },
    single(num, crc) {
        return Table[(num ^ crc) & 0xFF] ^ (crc >>> 8);
    },
    Table,
};
