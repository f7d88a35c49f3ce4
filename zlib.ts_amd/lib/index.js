// zlib.ts_amd: the reference's hot-path classes over the MI355X engine.
export { RawDeflate, CompressionType } from './RawDeflate.js';
export { RawInflate, BufferType } from './RawInflate.js';
export { RawInflateStream } from './RawInflateStream.js';
export { InflateStream } from './InflateStream.js';
export { CRC32 } from './CRC32.js';
export { Adler32 } from './Adler32.js';
export { GZip, GZipFlagsMask, GZipMagicNumber, GZipOperatingSystem } from './GZip.js';
export { GUnzip } from './GUnzip.js';
export { Deflate } from './Deflate.js';
export { Inflate } from './Inflate.js';
export { Zip, ZipCompressionMethod, ZipOperatingSystem, ZipFlags } from './Zip.js';
export { Unzip } from './Unzip.js';
import native from './native.js';
export const deviceCount = () => native.deviceCount();
export const version = () => native.version();
