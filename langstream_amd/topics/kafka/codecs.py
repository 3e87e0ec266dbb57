"""Record-batch compression codecs of the Kafka protocol (attributes bits 0-2):
1 gzip, 2 snappy (xerial-framed, as the Java client writes it, or raw), 3 lz4 (LZ4 frame
format, KIP-57), 4 zstd.

Producers of real deployments compress by default in many setups, so the consumer side
must decode every codec a broker may hand back.  No compression library beyond the
standard library (zlib) is available offline, so snappy and LZ4 are implemented here:
full decoders, and encoders that emit valid streams made of literal runs (correct,
uncompressed-size output -- the producer defaults to no compression anyway).  zstd is
rejected with a clear error (no decoder available).
"""
from __future__ import annotations

import struct
import zlib

NONE, GZIP, SNAPPY, LZ4, ZSTD = 0, 1, 2, 3, 4
NAMES = {"none": NONE, "gzip": GZIP, "snappy": SNAPPY, "lz4": LZ4, "zstd": ZSTD}


def codec_of(name) -> int:
    if name is None or name == "":
        return NONE
    if isinstance(name, int):
        return name
    try:
        return NAMES[str(name).lower()]
    except KeyError:
        raise ValueError(f"unknown compression.type {name}; known: {sorted(NAMES)}") from None


# ---------------------------------------------------------------- gzip
def gzip_compress(data: bytes) -> bytes:
    c = zlib.compressobj(6, zlib.DEFLATED, 31)
    return c.compress(data) + c.flush()


def gzip_decompress(data: bytes) -> bytes:
    return zlib.decompress(data, 47)   # gzip or zlib header


# ---------------------------------------------------------------- snappy
_XERIAL = b"\x82SNAPPY\x00"


def _uvarint(b: bytes, pos: int):
    v = shift = 0
    while True:
        c = b[pos]
        pos += 1
        v |= (c & 0x7F) << shift
        if c < 0x80:
            return v, pos
        shift += 7


def snappy_raw_decompress(data: bytes) -> bytes:
    n, pos = _uvarint(data, 0)
    out = bytearray()
    end = len(data)
    while pos < end:
        tag = data[pos]
        pos += 1
        t = tag & 3
        if t == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(data[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += data[pos:pos + ln]
            pos += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | data[pos]
            pos += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[pos:pos + 4], "little")
            pos += 4
        if off <= 0 or off > len(out):
            raise ValueError("corrupt snappy stream (bad copy offset)")
        start = len(out) - off
        if off >= ln:
            out += out[start:start + ln]
        else:                                  # overlapping copy
            for i in range(ln):
                out.append(out[start + i])
    if len(out) != n:
        raise ValueError(f"corrupt snappy stream ({len(out)} != {n} bytes)")
    return bytes(out)


def snappy_raw_compress(data: bytes) -> bytes:
    out = bytearray()
    n = len(data)
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            break
    pos = 0
    while pos < len(data):
        chunk = data[pos:pos + 65536]
        ln = len(chunk) - 1
        if ln < 60:
            out.append(ln << 2)
        elif ln < 256:
            out += bytes([60 << 2, ln])
        else:
            out += bytes([61 << 2]) + ln.to_bytes(2, "little")
        out += chunk
        pos += len(chunk)
    return bytes(out)


def snappy_decompress(data: bytes) -> bytes:
    if data[:8] != _XERIAL:
        return snappy_raw_decompress(data)
    pos, out = 16, bytearray()
    while pos + 4 <= len(data):
        ln = struct.unpack_from(">i", data, pos)[0]
        pos += 4
        out += snappy_raw_decompress(data[pos:pos + ln])
        pos += ln
    return bytes(out)


def snappy_compress(data: bytes) -> bytes:
    out = bytearray(_XERIAL + struct.pack(">ii", 1, 1))
    for i in range(0, max(len(data), 1), 32768):
        blk = snappy_raw_compress(data[i:i + 32768])
        out += struct.pack(">i", len(blk)) + blk
    return bytes(out)


# ---------------------------------------------------------------- lz4 (frame format)
_LZ4_MAGIC = 0x184D2204


def _xxh32(b: bytes) -> int:
    import xxhash
    return xxhash.xxh32(b, seed=0).intdigest()


def lz4_block_decompress(src: bytes, out: bytearray) -> None:
    pos, end = 0, len(src)
    while pos < end:
        token = src[pos]
        pos += 1
        lit = token >> 4
        if lit == 15:
            while True:
                c = src[pos]
                pos += 1
                lit += c
                if c != 255:
                    break
        out += src[pos:pos + lit]
        pos += lit
        if pos >= end:
            break
        off = src[pos] | (src[pos + 1] << 8)
        pos += 2
        ml = token & 15
        if ml == 15:
            while True:
                c = src[pos]
                pos += 1
                ml += c
                if c != 255:
                    break
        ml += 4
        if off <= 0 or off > len(out):
            raise ValueError("corrupt lz4 block (bad match offset)")
        start = len(out) - off
        if off >= ml:
            out += out[start:start + ml]
        else:
            for i in range(ml):
                out.append(out[start + i])


def lz4_decompress(data: bytes) -> bytes:
    if struct.unpack_from("<I", data, 0)[0] != _LZ4_MAGIC:
        raise ValueError("not an LZ4 frame")
    flg = data[4]
    pos = 6
    if flg & 0x08:
        pos += 8          # content size
    if flg & 0x01:
        pos += 4          # dictionary id
    pos += 1              # header checksum
    block_ck = bool(flg & 0x10)
    out = bytearray()
    while True:
        sz = struct.unpack_from("<I", data, pos)[0]
        pos += 4
        if sz == 0:
            break
        raw = bool(sz & 0x80000000)
        sz &= 0x7FFFFFFF
        blk = data[pos:pos + sz]
        pos += sz + (4 if block_ck else 0)
        if raw:
            out += blk
        else:
            lz4_block_decompress(blk, out)
    return bytes(out)


def lz4_compress(data: bytes) -> bytes:
    """LZ4 frame of uncompressed blocks (64 KB max block size, block independence)."""
    desc = bytes([0x60, 0x40])                        # version 01, block-independent; 64 KB blocks
    out = bytearray(struct.pack("<I", _LZ4_MAGIC) + desc + bytes([(_xxh32(desc) >> 8) & 0xFF]))
    for i in range(0, len(data), 65536):
        blk = data[i:i + 65536]
        out += struct.pack("<I", len(blk) | 0x80000000) + blk
    out += struct.pack("<I", 0)
    return bytes(out)


# ---------------------------------------------------------------- dispatch
def compress(codec: int, data: bytes) -> bytes:
    if codec == NONE:
        return data
    if codec == GZIP:
        return gzip_compress(data)
    if codec == SNAPPY:
        return snappy_compress(data)
    if codec == LZ4:
        return lz4_compress(data)
    raise ValueError("zstd compression is not available in this build")


def decompress(codec: int, data: bytes) -> bytes:
    if codec == GZIP:
        return gzip_decompress(data)
    if codec == SNAPPY:
        return snappy_decompress(data)
    if codec == LZ4:
        return lz4_decompress(data)
    if codec == ZSTD:
        raise ValueError("zstd-compressed record batches cannot be decoded in this build (no zstd library)")
    raise ValueError(f"unknown record batch compression codec {codec}")
