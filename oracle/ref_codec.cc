// TEST INFRASTRUCTURE ONLY — drives the UNMODIFIED reference LengthHeaderCodec
// (/root/reference/include/codec/LengthHeaderCodec.h over src/*.cc, compiled where they lie by
// `make ref`, never copied) behind a C ABI, so tests/golden/make_golden.py can record the reference's
// own encode/decode results as fixtures. Output goes to oracle/_ref/ (git-ignored).
#include "EventLoop.h"
#include "NetBuffer.h"
#include "codec/LengthHeaderCodec.h"

#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace {
annety::EventLoop* loop() {
  // Codec(EventLoop*) CHECKs a non-null loop (include/codec/Codec.h:22-25); encode/decode never use it.
  static thread_local annety::EventLoop* l = new annety::EventLoop();
  return l;
}

annety::LengthHeaderCodec::LENGTH_TYPE as_type(int t) {
  return static_cast<annety::LengthHeaderCodec::LENGTH_TYPE>(t);
}
}  // namespace

extern "C" {

// LengthHeaderCodec::encode (:146-201). Returns its rt; *out_len = bytes appended to the stream.
int ref_lhc_encode(int length_type, int64_t max_payload, const char* payload, size_t len, char* out, size_t cap,
                   size_t* out_len) {
  annety::LengthHeaderCodec codec(loop(), as_type(length_type), true, max_payload);
  annety::NetBuffer in, buff;
  in.append(payload, len);
  int rt = codec.encode(&in, &buff);
  size_t n = buff.readable_bytes();
  *out_len = n;
  if (n > cap) return -100;
  memcpy(out, buff.begin_read(), n);
  return rt;
}

// One LengthHeaderCodec::decode call (:71-137) on a stream holding `size` bytes. Returns its rt;
// *consumed = bytes it removed from the stream, *payload_len = bytes it appended to the payload.
int ref_lhc_decode(int length_type, int64_t max_payload, const char* stream, size_t size, char* payload, size_t cap,
                   size_t* payload_len, size_t* consumed) {
  annety::LengthHeaderCodec codec(loop(), as_type(length_type), true, max_payload);
  annety::NetBuffer buff, out;
  buff.append(stream, size);
  int rt = codec.decode(&buff, &out);
  *consumed = size - buff.readable_bytes();
  size_t n = out.readable_bytes();
  *payload_len = n;
  if (n > cap) return -100;
  memcpy(payload, out.begin_read(), n);
  return rt;
}

}  // extern "C"
