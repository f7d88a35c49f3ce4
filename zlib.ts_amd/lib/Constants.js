// Mirrors src/Constants.ts:1-24 of the reference (values used by the facade).
export const CompressionType = { NONE: 0, FIXED: 1, DYNAMIC: 2 };
export const BufferType = { BLOCK: 0, ADAPTIVE: 1 };
export const DefaultBufferSize = 0x8000;
export const DefaultDeflateBufferSize = 0x8000;
export const DefaultInflateBufferSize = 0x8000;
export const MaxBackwardLength = 32768;
export const MaxCopyLength = 258;
