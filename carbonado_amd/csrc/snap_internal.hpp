// snap_internal.hpp — the snappy framing pieces that host_stages.cpp's
// one-pass ECIES paths share with host_snap.cpp.  Library-internal: not part
// of the C-ABI or of host_stages.hpp's interface.
#pragma once

#include <cstddef>
#include <cstdint>

namespace chip {
namespace host {

inline constexpr size_t MAX_BLOCK = 65536;                                     // FrameEncoder's block
inline constexpr size_t MAX_COMPRESS_BLOCK = 32 + MAX_BLOCK + MAX_BLOCK / 6;  // max_compress_len(64 KiB)
inline constexpr uint8_t STREAM_ID[10] = {0xFF, 0x06, 0x00, 0x00, 's', 'N', 'a', 'P', 'p', 'Y'};

// CRC-32C of a block, masked as the framing format stores it
uint32_t crc_masked(const uint8_t *p, size_t n);
// snappy varint (a raw block's uncompressed length)
bool get_varint(const uint8_t *p, size_t n, uint64_t *v, size_t *used);
// raw snappy block decode into out[0..cap); false on corrupt input
bool decompress_raw(const uint8_t *src, size_t n, uint8_t *out, size_t cap, size_t *out_len);
// One chunk of the frame stream for len (<= MAX_BLOCK) input bytes: its 8-B
// header into hdr, its body (compressed into tmp, or the input itself when
// compression saves less than 1/8: FrameEncoder's rule) at *body; returns the
// body length.
size_t snap_block(const uint8_t *src, size_t len, uint8_t hdr[8], uint8_t *tmp, const uint8_t **body);

}  // namespace host
}  // namespace chip
