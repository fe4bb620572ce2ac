"""CPU restatement of the reference's SIMD-BP128 vector compression - TEST INFRASTRUCTURE ONLY (the checker for the
host encoder in csrc/host/storage.cpp and the device decoder hy_decode_simd_bp128; nothing in the product imports it).

Follows reference src/lib/storage/vector_compression/simd_bp128/:
  simd_bp128_compressor.cpp:13-120  meta blocks of 16 x 128 values, the last zero-padded; per meta block one 16-byte
                                    header word of the 16 blocks' bit widths (bits of the OR of the block's values),
                                    then the first ceil(values left / 128) blocks, `width` 16-byte words each
  simd_bp128_packing.cpp:22-157     Pack128Bit: value j of a block goes to 32-bit lane j % 4; per lane the values
                                    j % 4, j % 4 + 4, ... are concatenated low bits first, a value that does not fit the
                                    rest of a word continues at bit 0 of the same lane of the next word
Pinned by the reference's own test (src/test/storage/simd_bp128_test.cpp: bit sizes 1..32, 4,200-value sequences
cycling over [2^(b-1), 2^b - 1], decoded value == input).
"""
import numpy as np

BLOCK = 128
BLOCKS = 16
META = BLOCK * BLOCKS


def encode(values):
    """-> (words: np.uint32 array, 4 per 16-byte word, meta: list of header word indexes)."""
    v = np.asarray(values, dtype=np.uint64)
    n = len(v)
    out = []
    meta = []
    for m0 in range(0, n, META):
        meta.append(len(out) // 4)
        pend = np.zeros(META, dtype=np.uint64)
        part = v[m0:m0 + META]
        pend[:len(part)] = part
        widths = []
        for b in range(BLOCKS):
            acc = int(np.bitwise_or.reduce(pend[b * BLOCK:(b + 1) * BLOCK]))
            widths.append(acc.bit_length())
        header = np.frombuffer(bytes(widths), dtype=np.uint32)
        out.extend(int(x) for x in header)
        blocks = (len(part) + BLOCK - 1) // BLOCK
        for b in range(blocks):
            w = widths[b]
            if w == 0:  # pack_block: an all-zero block takes no words
                continue
            lanes = [[0] * w for _ in range(4)]
            for j in range(BLOCK):
                x = int(pend[b * BLOCK + j])
                lane, bit = j % 4, (j // 4) * w
                word, shift = bit // 32, bit % 32
                lanes[lane][word] |= (x << shift) & 0xFFFFFFFF
                if shift + w > 32:
                    lanes[lane][word + 1] |= x >> (32 - shift)
            for k in range(w):
                out.extend(lanes[lane][k] for lane in range(4))
    return np.array(out, dtype=np.uint32), meta


def decode(words, meta, n):
    """Every value, following the block / lane layout above."""
    words = np.asarray(words, dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        m, b, j = i // META, (i % META) // BLOCK, i % BLOCK
        h = meta[m]
        widths = np.frombuffer(words[4 * h:4 * h + 4].tobytes(), dtype=np.uint8)
        w = int(widths[b])
        if w == 0:
            continue
        word = h + 1 + int(widths[:b].astype(np.int64).sum())
        lane, bit = j % 4, (j // 4) * w
        k, shift = bit // 32, bit % 32
        x = int(words[4 * (word + k) + lane]) >> shift
        if shift + w > 32:
            x |= int(words[4 * (word + k + 1) + lane]) << (32 - shift)
        out[i] = x & ((1 << w) - 1)
    return out


def reference_sequence(bit_size, count=4200):
    """simd_bp128_test.cpp generate_sequence: min = 2^(b-1), max = 2^b - 1, cycling."""
    lo, hi = 1 << (bit_size - 1), (1 << bit_size) - 1
    span = hi - lo + 1
    return (lo + (np.arange(count, dtype=np.uint64) % span)).astype(np.uint64)
