// annety/Crc32c.h — drop-in replacement for the reference header include/Crc32c.h.
//
// Same namespace, class, method names, signatures and values as the reference
// (include/Crc32c.h:14-83; tables declared at :16-19 and defined in src/Crc32c.cc:20-92), so
// LengthHeaderCodec (include/codec/LengthHeaderCodec.h:107-121, 186-198) and ProtobufCodec
// (include/protobuf/ProtobufCodec.h:156-170, 235-247) compile unchanged against it. The six
// single-buffer methods stay inline on the calling thread, like the reference; the additive batch
// methods at the bottom hand whole batches of frames to the MI355X engine through the C-ABI in
// annety_crc.h (libannety_crc.so).
//
// Define ANNETY_CRC_NO_STRINGPIECE to use the header without annety's StringPiece.
#ifndef ANNETY_AMD_CRC32C_H
#define ANNETY_AMD_CRC32C_H

#include <stddef.h>
#include <stdint.h>

#include "annety_crc.h"

#ifndef ANNETY_CRC_NO_STRINGPIECE
#include "strings/StringPiece.h"
#endif

namespace annety {
namespace internal {
// Defined (constant-initialised from the polynomial) in libannety_crc.so: same symbols as
// src/Crc32c.cc so existing object files that reference them still link.
extern uint32_t crc32_table16[];
extern uint32_t crc32_table256[];
}  // namespace internal

class Crc32c {
 public:
#ifndef ANNETY_CRC_NO_STRINGPIECE
  static uint32_t crc32_short(const StringPiece& buff) { return crc32_short(buff.data(), buff.size()); }
  static uint32_t crc32_long(const StringPiece& buff) { return crc32_long(buff.data(), buff.size()); }
  static void crc32_update(uint32_t* crc, const StringPiece& buff) { crc32_update(crc, buff.data(), buff.size()); }
#endif

  // nibble-table variant (reference include/Crc32c.h:41-55); value identical to crc32_long
  static uint32_t crc32_short(const char* buff, size_t len) {
    uint32_t crc = 0xffffffffu;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
    while (len--) {
      const unsigned c = *p++;
      crc = internal::crc32_table16[(crc ^ (c & 0xfu)) & 0xfu] ^ (crc >> 4);
      crc = internal::crc32_table16[(crc ^ (c >> 4)) & 0xfu] ^ (crc >> 4);
    }
    return crc ^ 0xffffffffu;
  }

  // byte-table variant (reference include/Crc32c.h:58-69)
  static uint32_t crc32_long(const char* buff, size_t len) {
    uint32_t crc = 0xffffffffu;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
    while (len--) crc = internal::crc32_table256[(crc ^ *p++) & 0xffu] ^ (crc >> 8);
    return crc ^ 0xffffffffu;
  }

  // raw register, no init / final xor (reference include/Crc32c.h:71-82)
  static void crc32_update(uint32_t* crc, const char* buff, size_t len) {
    uint32_t c = *crc;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
    while (len--) c = internal::crc32_table256[(c ^ *p++) & 0xffu] ^ (c >> 8);
    *crc = c;
  }

  // ---- additive batch API (MI355X engine) ----
  // Device-resident fixed-length batch: crc of payload i = [d_base + i*stride, +len) into d_out[i].
  static int crc32_long_batch(const void* d_base, size_t n, size_t len, size_t stride, uint32_t* d_out,
                              void* hip_stream = nullptr) {
    return annety_crc32_batch_fixed(d_base, n, len, stride, d_out, hip_stream);
  }
  // Device-resident variable-length batch.
  static int crc32_long_batch(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                              uint32_t* d_out, void* hip_stream = nullptr) {
    return annety_crc32_batch_var(d_base, d_off, d_len, n, d_out, hip_stream);
  }
  // Device-resident variable-length batch whose payloads lie in [d_arena, d_arena + arena_bytes) and
  // mostly cover it (a received stream, a packed batch): one pass over the buffer.
  static int crc32_long_batch_arena(const void* d_arena, size_t arena_bytes, const uint64_t* d_off,
                                    const uint32_t* d_len, size_t n, uint32_t* d_out, void* hip_stream = nullptr) {
    return annety_crc32_batch_var_arena(d_arena, arena_bytes, d_off, d_len, n, d_out, hip_stream);
  }
  // crc32_update over a batch: d_state[i] advanced over fragment i (fixed stride, or offsets/lengths).
  static int crc32_update_batch(uint32_t* d_state, const void* d_base, size_t n, size_t len, size_t stride,
                                void* hip_stream = nullptr) {
    return annety_crc32_update_batch_fixed(d_state, d_base, n, len, stride, hip_stream);
  }
  static int crc32_update_batch(uint32_t* d_state, const void* d_base, const uint64_t* d_off, const uint32_t* d_len,
                                size_t n, void* hip_stream = nullptr) {
    return annety_crc32_update_batch_var(d_state, d_base, d_off, d_len, n, hip_stream);
  }
  // Host-memory batch (staged H2D -> kernel -> D2H); synchronous.
  static int crc32_long_batch_host(const void* h_base, size_t n, size_t len, size_t stride, uint32_t* h_out) {
    return annety_crc32_batch_fixed_host(h_base, n, len, stride, h_out);
  }
  static uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return annety_crc32_combine(crc_a, crc_b, len_b);
  }
};

}  // namespace annety

#endif  // ANNETY_AMD_CRC32C_H
