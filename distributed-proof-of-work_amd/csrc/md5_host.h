// md5_host.h -- host MD5 used by the planner (midstates) and hit verification.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace dpow {
void md5_compress(uint32_t st[4], const uint32_t M[16]);
void md5_digest(const uint8_t *msg, size_t len, uint8_t out[16]);
uint32_t digest_trailing_zero_nibbles(const uint8_t d[16]);
uint32_t load_le32(const uint8_t *p);
}  // namespace dpow
