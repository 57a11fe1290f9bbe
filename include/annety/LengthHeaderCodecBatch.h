// annety/LengthHeaderCodecBatch.h — batched counterpart of annety::LengthHeaderCodec for the MI355X
// engine.
//
// The reference codec (include/codec/LengthHeaderCodec.h:37-231) frames one message per call:
//   [length: T bytes big-endian, T = 1/2/4/8, value = payload + 4][payload][crc32(payload): 4 bytes BE]
// and Codec::recv (include/codec/Codec.h:52-76) loops decode() over a receive buffer until it returns
// 0 (incomplete) or -1 (invalid length or checksum: the connection is shut down). This class does the
// same work for a whole buffer or a whole batch at once, with every CRC on the GPU:
//   decode side: locate() walks the headers on the host (a serial chain of a few ns per frame),
//                verify() checks every located frame's trailer on the device in one launch sequence,
//                recv_outcome() turns the verdicts into exactly what the recv loop would have done;
//   encode side: plan() applies encode()'s length checks and lays the frames out back to back,
//                encode() writes header, payload copy and trailer of every frame on the device.
// Checksums are always enabled (the checksum-less codec has no device work).
#ifndef ANNETY_AMD_LENGTH_HEADER_CODEC_BATCH_H
#define ANNETY_AMD_LENGTH_HEADER_CODEC_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "annety_crc.h"

namespace annety {

class LengthHeaderCodecBatch {
 public:
  enum LENGTH_TYPE { kLengthType8 = 1, kLengthType16 = 2, kLengthType32 = 4, kLengthType64 = 8 };

  // Same defaults as LengthHeaderCodec's constructor (:48-51); max_payload <= 0 means unlimited.
  explicit LengthHeaderCodecBatch(LENGTH_TYPE length_type = kLengthType32, int64_t max_payload = 64 * 1024 * 1024)
      : length_type_(length_type), max_payload_(max_payload) {}

  // Complete frames found in a receive buffer (offsets relative to it).
  struct Frames {
    std::vector<uint64_t> payload_off;
    std::vector<uint32_t> payload_len;
    size_t consumed = 0;          // bytes of the frames found
    bool invalid_length = false;  // the walk stopped on decode()'s length check (:102-106)
  };

  // Host header walk (annety_lhc_parse). Returns 0 or a negative ANNETY_CRC_E* status.
  int locate(const char* buff, size_t size, Frames* frames, size_t max_frames = (size_t)-1) const {
    const size_t fit = size / ((size_t)length_type_ + 4) + 1;
    const size_t cap = max_frames < fit ? max_frames : fit;
    frames->payload_off.resize(cap);
    frames->payload_len.resize(cap);
    size_t k = 0;
    const int st = annety_lhc_parse(buff, size, (int)length_type_, max_payload_, frames->payload_off.data(),
                                    frames->payload_len.data(), cap, &k, &frames->consumed);
    frames->payload_off.resize(k);
    frames->payload_len.resize(k);
    frames->invalid_length = st == 1;
    return st < 0 ? st : ANNETY_CRC_OK;
  }

  // Device checksum test of n located frames (device pointers): d_ok[i] = trailer matches.
  static int verify(const void* d_buff, const uint64_t* d_off, const uint32_t* d_len, size_t n, uint8_t* d_ok,
                    uint32_t* d_digest = nullptr, void* hip_stream = nullptr) {
    return annety_lhc_verify_batch(d_buff, d_off, d_len, n, d_ok, d_digest, hip_stream);
  }

  // Codec::recv's outcome from locate() and the verdicts (host copy of d_ok): frames [0, *delivered)
  // are the ones decode() returned 1 for, *consumed the bytes they took; returns the decode() result
  // that ended the loop: -1 (bad checksum or invalid length) or 0.
  int recv_outcome(const Frames& frames, const uint8_t* ok, size_t* delivered, size_t* consumed) const {
    const size_t n = frames.payload_off.size();
    for (size_t i = 0; i < n; i++) {
      if (!ok[i]) {
        *delivered = i;
        *consumed = (size_t)frames.payload_off[i] - (size_t)length_type_;
        return -1;
      }
    }
    *delivered = n;
    *consumed = frames.consumed;
    return frames.invalid_length ? -1 : 0;
  }

  // encode()'s per-payload decision (:169-176: 1, 0 for an empty payload, -1 above max_payload) and the
  // output offset of every frame, accepted frames packed back to back. Host arrays of n entries.
  int plan(const uint32_t* len, size_t n, uint64_t* frame_off, int8_t* rt, uint64_t* total) const {
    return annety_lhc_encode_plan(len, n, (int)length_type_, max_payload_, frame_off, rt, total);
  }

  // Device encode of the accepted payloads (offsets from plan() copied to the device).
  int encode(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len, size_t n, void* d_dst,
             const uint64_t* d_frame_off, void* hip_stream = nullptr) const {
    return annety_lhc_encode_batch(d_src, d_src_off, d_len, n, (int)length_type_, max_payload_, d_dst, d_frame_off,
                                   hip_stream);
  }

  LENGTH_TYPE length_type() const { return length_type_; }
  int64_t max_payload() const { return max_payload_; }

 private:
  LENGTH_TYPE length_type_;
  int64_t max_payload_;
};

}  // namespace annety

#endif  // ANNETY_AMD_LENGTH_HEADER_CODEC_BATCH_H
