"""The hash loop's per-candidate D-word test, restated on the host with the planner's
launch fields (dpow_diag_dword_test): its one-compare prefilter plus the rare path's
nibble mask must equal the reference's hex-suffix rule on the D word
(hasNumZeroesSuffix, worker.go:246-256) for every N, in every layout."""
import random

import pytest

import distpow
from distpow._lib import lib

IV_D = 0x10325476  # RFC 1321 chaining value D entering the first block


def _tz_dword(D):
    """Trailing '0' hex characters of the digest's last four bytes (D little-endian)."""
    h = D.to_bytes(4, "little").hex()
    return len(h) - len(h.rstrip("0"))


def _iv_d(nonce):
    iv, words, nblk = distpow.plan_candidate(nonce, 0, 0, 0)
    return iv[3], nblk


def _dvals(rnd):
    vals = [0, 1, 0xFFFFFFFF, 0x80000000]
    for z in range(9):  # D with exactly z trailing zero nibbles (hex order), and neighbours
        for _ in range(40):
            h = list(rnd.getrandbits(32).to_bytes(4, "little").hex())
            for j in range(z):
                h[7 - j] = "0"
            if z < 8 and h[7 - z] == "0":
                h[7 - z] = "1"
            vals.append(int.from_bytes(bytes.fromhex("".join(h)), "little"))
    return vals


@pytest.mark.parametrize("nlen", [0, 4, 23, 51, 60, 70, 129])
def test_dword_test_equals_hex_suffix_rule(nlen):
    rnd = random.Random(nlen)
    nonce = bytes(rnd.randrange(256) for _ in range(nlen)) if nlen != 4 else bytes([1, 2, 3, 4])
    iv_d, nblk = _iv_d(nonce)
    for D in _dvals(rnd):
        # one final block: the chaining value is fixed; two: any per-candidate value
        ivs = [iv_d] if nblk == 1 else [iv_d, rnd.getrandbits(32)]
        for iv in ivs:
            state = (D - iv) & 0xFFFFFFFF
            for ntz in list(range(0, 11)) + [16, 32]:
                got = lib().dpow_diag_dword_test(nonce, len(nonce), ntz, 0, iv, state)
                assert got in (0, 1), got
                assert got == int(_tz_dword(D) >= min(ntz, 8)), (nlen, hex(D), ntz)
