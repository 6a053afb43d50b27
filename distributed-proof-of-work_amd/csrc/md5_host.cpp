// md5_host.cpp -- host-side MD5 of the product: midstates for nonces longer
// than one block, and the re-verification of every kernel hit
// (north star: "verified by recomputing MD5 on the host").  Word-oriented
// compression over the same constant tables the kernel uses.
#include <string.h>

#include "dpow_common.h"
#include "md5_host.h"

namespace dpow {

static inline uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

void md5_compress(uint32_t st[4], const uint32_t M[16]) {
    uint32_t x[4] = {st[0], st[1], st[2], st[3]};
    for (int i = 0; i < 64; ++i) {
        const int ai = (64 - i) % 4, bi = (ai + 1) % 4, ci = (ai + 2) % 4, di = (ai + 3) % 4;
        const uint32_t b = x[bi], c = x[ci], d = x[di];
        uint32_t f;
        switch (i >> 4) {
            case 0: f = (b & c) | (~b & d); break;
            case 1: f = (b & d) | (c & ~d); break;
            case 2: f = b ^ c ^ d; break;
            default: f = c ^ (b | ~d); break;
        }
        x[ai] = b + rol(x[ai] + f + kMd5K[i] + M[md5_word(i)], md5_shift(i));
    }
    for (int w = 0; w < 4; ++w) st[w] += x[w];
}

uint32_t load_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

void md5_digest(const uint8_t *msg, size_t len, uint8_t out[16]) {
    uint32_t st[4] = {kMd5IV[0], kMd5IV[1], kMd5IV[2], kMd5IV[3]};
    uint32_t M[16];
    size_t off = 0;
    for (; off + 64 <= len; off += 64) {
        for (int w = 0; w < 16; ++w) M[w] = load_le32(msg + off + 4 * w);
        md5_compress(st, M);
    }
    uint8_t tail[128];
    memset(tail, 0, sizeof tail);
    const size_t rem = len - off;
    if (rem) memcpy(tail, msg + off, rem);
    tail[rem] = 0x80;
    const size_t tlen = rem + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)len * 8u;
    for (int j = 0; j < 8; ++j) tail[tlen - 8 + j] = (uint8_t)(bits >> (8 * j));
    for (size_t b = 0; b < tlen; b += 64) {
        for (int w = 0; w < 16; ++w) M[w] = load_le32(tail + b + 4 * w);
        md5_compress(st, M);
    }
    for (int w = 0; w < 4; ++w)
        for (int j = 0; j < 4; ++j) out[4 * w + j] = (uint8_t)(st[w] >> (8 * j));
}

uint32_t digest_trailing_zero_nibbles(const uint8_t d[16]) {
    // hex string = d[0] hi, d[0] lo, ..., d[15] hi, d[15] lo; count '0' from the end.
    uint32_t n = 0;
    for (int i = 15; i >= 0; --i) {
        if ((d[i] & 0x0F) != 0) return n;
        ++n;
        if ((d[i] & 0xF0) != 0) return n;
        ++n;
    }
    return n;
}

}  // namespace dpow
