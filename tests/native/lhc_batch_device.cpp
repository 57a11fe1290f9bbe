// Device side of include/annety/LengthHeaderCodecBatch.h, through the C++ class alone (tests/test_lhc.py runs it on
// the GPU): plan() + encode() on the device for a batch of payloads (empty ones and ones above max_payload among
// them, which encode() rejects, LengthHeaderCodec.h:169-176), every frame checked byte by byte on the host against
// the drop-in's host Crc32c; then locate() + verify() on the device + recv_outcome() over the encoded stream, which
// must deliver every frame, and again with one byte of frame k flipped, which must stop Codec::recv at frame k
// (include/codec/Codec.h:52-76). Built by annety_amd/build.py next to the library.
// Usage: lhc_batch_device T n seed   (prints "ok <accepted frames> <stream bytes>")
#define ANNETY_CRC_NO_STRINGPIECE
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "annety/Crc32c.h"
#include "annety/LengthHeaderCodecBatch.h"

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("fail %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(2);                                                                 \
    }                                                                               \
  } while (0)
#define EXPECT(c, ...)             \
  do {                             \
    if (!(c)) {                    \
      std::printf("fail: ");       \
      std::printf(__VA_ARGS__);    \
      std::printf("\n");           \
      std::exit(1);                \
    }                              \
  } while (0)

static uint64_t g_state;
static uint32_t rnd() {
  g_state = g_state * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(g_state >> 33);
}

template <class T>
static T* to_device(const std::vector<T>& h) {
  T* d = nullptr;
  CK(hipMalloc(&d, h.size() * sizeof(T) + 16));
  if (!h.empty()) CK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  return d;
}

int main(int argc, char** argv) {
  if (argc != 4) return 3;
  const int T = std::atoi(argv[1]);
  const size_t n = (size_t)std::atoll(argv[2]);
  g_state = (uint64_t)std::atoll(argv[3]);
  // a length field of T bytes holds length + 4 (:188-198), which decode() reads back signed (peek_int8/16,
  // include/NetBuffer.h): keep it below 2^(8T-1) so that the receive side can parse every frame written
  const int64_t maxp = T == 1 ? 100 : (T == 2 ? 30000 : 100000);
  typedef annety::LengthHeaderCodecBatch Codec;
  const Codec codec((Codec::LENGTH_TYPE)T, maxp);

  // payloads packed back to back after a 3-byte lead, lengths 0 .. 1.2 max_payload (some rejected, some empty)
  std::vector<uint32_t> len(n);
  std::vector<uint64_t> src_off(n);
  uint64_t pos = 3;
  for (size_t i = 0; i < n; i++) {
    const uint32_t r = rnd();
    len[i] = r % 17 == 0 ? 0u : (uint32_t)(r % (uint32_t)(maxp + maxp / 5));
    src_off[i] = pos;
    pos += len[i];
  }
  std::vector<char> src(pos + 8);
  for (auto& c : src) c = (char)rnd();

  std::vector<uint64_t> frame_off(n);
  std::vector<int8_t> rt(n);
  uint64_t total = 0;
  EXPECT(codec.plan(len.data(), n, frame_off.data(), rt.data(), &total) == 0, "plan");
  char* d_src = to_device(src);
  uint64_t* d_src_off = to_device(src_off);
  uint32_t* d_len = to_device(len);
  uint64_t* d_frame_off = to_device(frame_off);
  char* d_dst = nullptr;
  CK(hipMalloc(&d_dst, total + 16));
  CK(hipMemset(d_dst, 0xA5, total + 16));
  EXPECT(codec.encode(d_src, d_src_off, d_len, n, d_dst, d_frame_off) == 0, "encode");
  CK(hipDeviceSynchronize());
  std::vector<char> dst(total);
  if (total) CK(hipMemcpy(dst.data(), d_dst, total, hipMemcpyDeviceToHost));

  // every accepted frame: header (length + 4, big-endian, low T bytes), payload, trailer; nothing for the others
  size_t accepted = 0;
  uint64_t at = 0;
  for (size_t i = 0; i < n; i++) {
    const int8_t want_rt = len[i] == 0 ? 0 : ((int64_t)len[i] > maxp ? -1 : 1);
    EXPECT(rt[i] == want_rt, "plan rt[%zu] = %d, want %d", i, rt[i], want_rt);
    if (rt[i] != 1) continue;
    EXPECT(frame_off[i] == at, "frame %zu at %llu, want %llu", i, (unsigned long long)frame_off[i],
           (unsigned long long)at);
    const unsigned char* f = reinterpret_cast<const unsigned char*>(dst.data() + at);
    const uint64_t hdr = (uint64_t)len[i] + 4;
    for (int b = 0; b < T; b++)
      EXPECT(f[b] == (unsigned char)(hdr >> (8 * (T - 1 - b))), "frame %zu header byte %d", i, b);
    for (uint32_t b = 0; b < len[i]; b++)
      EXPECT(f[T + b] == (unsigned char)src[src_off[i] + b], "frame %zu payload byte %u", i, b);
    const uint32_t crc = annety::Crc32c::crc32_long(src.data() + src_off[i], len[i]);
    for (int b = 0; b < 4; b++)
      EXPECT(f[T + len[i] + b] == (unsigned char)(crc >> (24 - 8 * b)), "frame %zu trailer byte %d", i, b);
    at += (uint64_t)T + len[i] + 4;
    accepted++;
  }
  EXPECT(at == total, "stream %llu bytes, plan %llu", (unsigned long long)at, (unsigned long long)total);

  // the receive side over the encoded stream: every frame delivered, then a flipped byte in frame k stops it there.
  // decode() checks the length field (payload + 4) against max_payload (:100-106) where encode() checked the payload
  // (:169-176), so the receiver takes max_payload + 4 to accept every frame the sender wrote
  const Codec rx((Codec::LENGTH_TYPE)T, maxp + 4);
  Codec::Frames fr;
  EXPECT(rx.locate(dst.data(), dst.size(), &fr) == 0, "locate");
  EXPECT(fr.payload_off.size() == accepted && fr.consumed == total, "located %zu frames", fr.payload_off.size());
  uint64_t* d_off = to_device(fr.payload_off);
  uint32_t* d_flen = to_device(fr.payload_len);
  uint8_t* d_ok = nullptr;
  uint32_t* d_dig = nullptr;
  CK(hipMalloc(&d_ok, accepted + 16));
  CK(hipMalloc(&d_dig, 4 * accepted + 16));
  for (int pass = 0; pass < 2; pass++) {
    size_t k = accepted / 2;
    while (pass == 1 && k < accepted && fr.payload_len[k] == 0) k++;  // (every accepted frame has a payload byte)
    if (pass == 1) {
      EXPECT(k < accepted, "no frame to corrupt");
      const uint64_t b = fr.payload_off[k] + fr.payload_len[k] / 2;
      dst[b] ^= 0x10;
      CK(hipMemcpy(d_dst + b, dst.data() + b, 1, hipMemcpyHostToDevice));
    }
    CK(hipMemset(d_ok, 0x7F, accepted + 16));
    EXPECT(Codec::verify(d_dst, d_off, d_flen, accepted, d_ok, d_dig) == 0, "verify");
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> ok(accepted);
    std::vector<uint32_t> dig(accepted);
    if (accepted) {
      CK(hipMemcpy(ok.data(), d_ok, accepted, hipMemcpyDeviceToHost));
      CK(hipMemcpy(dig.data(), d_dig, 4 * accepted, hipMemcpyDeviceToHost));
    }
    for (size_t i = 0; i < accepted; i++) {
      const uint32_t crc = annety::Crc32c::crc32_long(dst.data() + fr.payload_off[i], fr.payload_len[i]);
      EXPECT(dig[i] == crc, "pass %d digest %zu", pass, i);
      EXPECT(ok[i] == (pass == 1 && i == k ? 0 : 1), "pass %d verdict %zu = %d", pass, i, ok[i]);
    }
    size_t delivered = 0, consumed = 0;
    const int r = rx.recv_outcome(fr, ok.data(), &delivered, &consumed);
    if (pass == 0) {
      EXPECT(r == 0 && delivered == accepted && consumed == total, "recv %d %zu %zu", r, delivered, consumed);
    } else {
      EXPECT(r == -1 && delivered == k && consumed == fr.payload_off[k] - (uint64_t)T, "recv after flip %d %zu %zu", r,
             delivered, consumed);
    }
  }
  std::printf("ok %zu %llu\n", accepted, (unsigned long long)total);
  return 0;
}
