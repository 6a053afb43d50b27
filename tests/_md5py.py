"""Tiny pure-Python MD5 compression (RFC 1321) for midstate checks in tests -- TEST INFRASTRUCTURE."""
import math
import struct

K = [int(abs(math.sin(i + 1)) * (1 << 32)) & 0xFFFFFFFF for i in range(64)]
S = [7, 12, 17, 22] * 4 + [5, 9, 14, 20] * 4 + [4, 11, 16, 23] * 4 + [6, 10, 15, 21] * 4
IV = (0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476)


def _rol(x, s):
    x &= 0xFFFFFFFF
    return ((x << s) | (x >> (32 - s))) & 0xFFFFFFFF


def compress(state, words):
    a, b, c, d = state
    for i in range(64):
        if i < 16:
            f, g = (b & c) | (~b & d), i
        elif i < 32:
            f, g = (d & b) | (~d & c), (5 * i + 1) % 16
        elif i < 48:
            f, g = b ^ c ^ d, (3 * i + 5) % 16
        else:
            f, g = c ^ (b | (~d & 0xFFFFFFFF)), (7 * i) % 16
        a, d, c, b = d, c, b, (b + _rol(a + f + K[i] + words[g], S[i])) & 0xFFFFFFFF
    return tuple((x + y) & 0xFFFFFFFF for x, y in zip(state, (a, b, c, d)))


def padded_blocks(msg: bytes):
    ml = len(msg)
    m = msg + b"\x80" + b"\x00" * ((55 - ml) % 64) + struct.pack("<Q", ml * 8)
    return [list(struct.unpack("<16I", m[i:i + 64])) for i in range(0, len(m), 64)]


def digest_from_state(state) -> bytes:
    return struct.pack("<4I", *state)
