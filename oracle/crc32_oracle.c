/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle for annety's checksum path.
 *
 * This file is the parity checker for the MI355X engine. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product (libannety_crc.so) never links it.
 *
 * It restates, in plain C, the algorithm of the reference's checksum path:
 *   - tables          : src/Crc32c.cc:20-25 (crc32_table16), src/Crc32c.cc:27-92 (crc32_table256)
 *                       generated here from the reflected IEEE polynomial 0xEDB88320 instead of copied;
 *   - crc32_long      : include/Crc32c.h:58-69   (byte-wise, 256-entry table)
 *   - crc32_short     : include/Crc32c.h:41-55   (two nibble steps per byte, 16-entry table)
 *   - crc32_update    : include/Crc32c.h:71-82   (raw register, no init / no final xor)
 * plus batch drivers and helpers used by the tests (combine, LCG payload generator of SURVEY.md §8c).
 *
 * Parity is pinned: tests/test_oracle.py checks every function here against the compiled reference
 * (oracle/_ref, built by oracle/Makefile from /root/reference/src/Crc32c.cc) through the golden
 * fixtures in tests/golden/, and against Python's zlib.crc32.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_POLY 0xEDB88320u

static uint32_t g_t256[256];
static uint32_t g_t16[16];
static int g_ready = 0;

/* src/Crc32c.cc:27-92: entry i = 8 reflected shift/xor rounds of i. */
static void oracle_build(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (ORACLE_POLY & (0u - (c & 1u)));
    g_t256[i] = c;
  }
  /* src/Crc32c.cc:20-25: the 16-entry table equals table256[16*i]. */
  for (uint32_t i = 0; i < 16; i++) g_t16[i] = g_t256[16 * i];
  g_ready = 1;
}

static inline void ensure(void) {
  if (!g_ready) oracle_build();
}

void oracle_tables(uint32_t* t256, uint32_t* t16) {
  ensure();
  memcpy(t256, g_t256, sizeof g_t256);
  memcpy(t16, g_t16, sizeof g_t16);
}

/* include/Crc32c.h:58-69 */
uint32_t oracle_crc32_long(const unsigned char* buf, size_t len) {
  ensure();
  uint32_t crc = 0xFFFFFFFFu;
  while (len--) crc = g_t256[(crc ^ *buf++) & 0xff] ^ (crc >> 8);
  return crc ^ 0xFFFFFFFFu;
}

/* include/Crc32c.h:41-55 (the reference uses `char c; c >> 4` — masked with & 0xf, so the
 * signedness of char does not change the value). */
uint32_t oracle_crc32_short(const unsigned char* buf, size_t len) {
  ensure();
  uint32_t crc = 0xFFFFFFFFu;
  while (len--) {
    unsigned c = *buf++;
    crc = g_t16[(crc ^ (c & 0xf)) & 0xf] ^ (crc >> 4);
    crc = g_t16[(crc ^ (c >> 4)) & 0xf] ^ (crc >> 4);
  }
  return crc ^ 0xFFFFFFFFu;
}

/* include/Crc32c.h:71-82 */
void oracle_crc32_update(uint32_t* crc, const unsigned char* buf, size_t len) {
  ensure();
  uint32_t c = *crc;
  while (len--) c = g_t256[(c ^ *buf++) & 0xff] ^ (c >> 8);
  *crc = c;
}

/* Raw-register shift by n zero bytes (the linear map x^(8n) mod P). Used by combine. */
static uint32_t gf2_times(const uint32_t* mat, uint32_t vec) {
  uint32_t sum = 0;
  for (int i = 0; vec; i++, vec >>= 1)
    if (vec & 1) sum ^= mat[i];
  return sum;
}
static void gf2_square(uint32_t* sq, const uint32_t* mat) {
  for (int n = 0; n < 32; n++) sq[n] = gf2_times(mat, mat[n]);
}
uint32_t oracle_shift_bytes(uint32_t c, uint64_t nbytes) {
  /* operator for one zero bit: column i = image of bit i */
  uint32_t odd[32], even[32];
  if (nbytes == 0 || c == 0) return c;
  odd[0] = ORACLE_POLY;
  for (int i = 1; i < 32; i++) odd[i] = 1u << (i - 1);
  gf2_square(even, odd); /* 2 bits */
  gf2_square(odd, even); /* 4 bits */
  /* odd = 4 bits; square once more gives one byte in even, then walk the bits of nbytes */
  for (;;) {
    gf2_square(even, odd); /* 8 bits, 32 bits, ... */
    if (nbytes & 1) c = gf2_times(even, c);
    nbytes >>= 1;
    if (!nbytes) break;
    gf2_square(odd, even);
    if (nbytes & 1) c = gf2_times(odd, c);
    nbytes >>= 1;
    if (!nbytes) break;
  }
  return c;
}

/* crc(A||B) from crc(A), crc(B), |B|  (final, conditioned values; zlib's identity) */
uint32_t oracle_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  return oracle_shift_bytes(crc1, len2) ^ crc2;
}

/* Batch drivers: payload i at base + i*stride (fixed) or base + off[i] (variable). */
void oracle_crc32_batch_fixed(const unsigned char* base, size_t n, size_t len, size_t stride, uint32_t* out) {
  for (size_t i = 0; i < n; i++) out[i] = oracle_crc32_long(base + i * stride, len);
}
void oracle_crc32_batch_var(const unsigned char* base, const uint64_t* off, const uint32_t* len, size_t n,
                            uint32_t* out) {
  for (size_t i = 0; i < n; i++) out[i] = oracle_crc32_long(base + off[i], len[i]);
}

/* Payload-parallel batch over T host threads (one worker per core, mirroring annety's one loop per
 * thread, src/EventLoopPool.cc:55-66). Used only for the cpu_baseline leg of bench.py. */
typedef struct {
  const unsigned char* base;
  size_t lo, hi, len, stride;
  uint32_t* out;
} job_t;
static void* worker(void* p) {
  job_t* j = (job_t*)p;
  for (size_t i = j->lo; i < j->hi; i++) j->out[i] = oracle_crc32_long(j->base + i * j->stride, j->len);
  return NULL;
}
int oracle_crc32_batch_fixed_mt(const unsigned char* base, size_t n, size_t len, size_t stride, uint32_t* out,
                                int threads) {
  ensure();
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  job_t jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t].base = base;
    jobs[t].lo = n * (size_t)t / threads;
    jobs[t].hi = n * (size_t)(t + 1) / threads;
    jobs[t].len = len;
    jobs[t].stride = stride;
    jobs[t].out = out;
    if (pthread_create(&tid[t], NULL, worker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  return 0;
}

/* SURVEY.md §8c seeded payload generator: s = s*6364136223846793005 + 1442695040888963407 (mod 2^64),
 * byte = s >> 56, filled sequentially across payloads. Returns the final state so callers can continue. */
uint64_t oracle_lcg_fill(unsigned char* buf, size_t nbytes, uint64_t seed) {
  uint64_t s = seed;
  for (size_t i = 0; i < nbytes; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    buf[i] = (unsigned char)(s >> 56);
  }
  return s;
}

/* ---- LengthHeaderCodec frames (include/codec/LengthHeaderCodec.h), checksum enabled ----
 * frame = [length: T bytes BE (signed, NetBuffer::peek_intN / append_intN, include/NetBuffer.h:38-125)]
 *         [payload: length-4 bytes][crc32(payload): 4 bytes BE (append_int32 / peek_uint32 :18-23)] */

/* append_intT(x) stores the low T bytes of x big-endian (the implicit narrowing to int8/16/32_t). */
static void put_be(unsigned char* p, int T, uint64_t x) {
  for (int b = 0; b < T; b++) p[b] = (unsigned char)(x >> (8 * (T - 1 - b)));
}

/* LengthHeaderCodec::encode (:146-201). Returns its rt (1 ok, 0 empty payload -> nothing written,
 * -1 length > max_payload); *out_len = bytes appended. `out` must hold T + len + 4 bytes. */
int oracle_lhc_encode(int T, int64_t max_payload, const unsigned char* payload, size_t len, unsigned char* out,
                      size_t* out_len) {
  *out_len = 0;
  if (len == 0) return 0;                                   /* :169-171 */
  if (max_payload > 0 && (int64_t)len > max_payload) return -1; /* :172-176 (min check is len < 0) */
  put_be(out, T, (uint64_t)len + 4);                        /* :179 set_buff_length(length + 4) */
  memcpy(out + T, payload, len);                            /* :180 */
  put_be(out + T + len, 4, oracle_crc32_long(payload, len)); /* :185-196 long/short agree */
  *out_len = (size_t)T + len + 4;
  return 1;
}

/* One LengthHeaderCodec::decode call (:71-137) on `size` readable bytes. Returns its rt (1 frame,
 * 0 incomplete, -1 invalid length or checksum); on 1, the payload is stream[*payload_off, +*payload_len)
 * and *consumed = T + length bytes are removed. */
int oracle_lhc_decode(int T, int64_t max_payload, const unsigned char* s, size_t size, size_t* payload_off,
                      size_t* payload_len, size_t* consumed) {
  *payload_off = *payload_len = *consumed = 0;
  if (size < (size_t)T) return 0;                           /* :100 */
  uint64_t u = 0;
  for (int b = 0; b < T; b++) u = (u << 8) | s[b];
  int64_t length;                                           /* :75-96 signed peek */
  switch (T) {
    case 1: length = (int8_t)u; break;
    case 2: length = (int16_t)u; break;
    case 4: length = (int32_t)u; break;
    default: length = (int64_t)u; break;
  }
  if (length < 4 || (max_payload > 0 && length > max_payload)) return -1; /* :102-106, min_payload = 4 */
  if (size - (size_t)T < (uint64_t)length) return 0;       /* :107 */
  const unsigned char* tr = s + T + length - 4;            /* :112 */
  uint32_t want = ((uint32_t)tr[0] << 24) | ((uint32_t)tr[1] << 16) | ((uint32_t)tr[2] << 8) | tr[3];
  if (oracle_crc32_long(s + T, (size_t)length - 4) != want) return -1; /* :113-132 */
  *payload_off = (size_t)T;
  *payload_len = (size_t)length - 4;
  *consumed = (size_t)T + (size_t)length;
  return 1;
}

/* Variable batches over T threads (payload-parallel, as above): digests (crc32_long) or, with
 * `update` set, crc32_update of out[i] in place (include/Crc32c.h:71-82). Test checker for the
 * full-size variable-length parity cases (BASELINE config 3) and the cpu_baseline leg. */
typedef struct {
  const unsigned char* base;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint32_t* out;
  int update;
} vjob_t;
static void* vworker(void* p) {
  vjob_t* j = (vjob_t*)p;
  for (size_t i = j->lo; i < j->hi; i++) {
    if (j->update)
      oracle_crc32_update(&j->out[i], j->base + j->off[i], j->len[i]);
    else
      j->out[i] = oracle_crc32_long(j->base + j->off[i], j->len[i]);
  }
  return NULL;
}
int oracle_crc32_batch_var_mt(const unsigned char* base, const uint64_t* off, const uint32_t* len, size_t n,
                              uint32_t* out, int update, int threads) {
  ensure();
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  vjob_t jobs[256];
  for (int t = 0; t < threads; t++) {
    vjob_t j = {base, off, len, n * (size_t)t / threads, n * (size_t)(t + 1) / threads, out, update};
    jobs[t] = j;
    if (pthread_create(&tid[t], NULL, vworker, &jobs[t]) != 0) {
      for (int k = 0; k < t; k++) pthread_join(tid[k], NULL);
      return -1;
    }
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
  return 0;
}

/* ---- ProtobufCodec framing (include/protobuf/ProtobufCodec.h), checksum enabled ----
 * Same frame layout as LengthHeaderCodec with length_type() = kLengthType32 (:260-263),
 * min_payload() = header_length() 4 + 2 + checksum_length() 4 = 10 (:279-283) and
 * max_payload() = 64 MiB, always enforced (:273-277). Parity is unpinned against the reference
 * itself (its header needs libprotobuf, absent here); these restate :127-173 and :206-247. */
#define PBC_MIN_PAYLOAD 10
#define PBC_MAX_PAYLOAD (64ll * 1024 * 1024)

/* ProtobufCodec::encode (:206-247): 0 for an empty payload, -1 for len < 10 - 4 or len > 64 MiB. */
int oracle_pbc_encode(const unsigned char* payload, size_t len, unsigned char* out, size_t* out_len) {
  *out_len = 0;
  if (len == 0) return 0;                                                              /* :223-225 */
  if ((int64_t)len < PBC_MIN_PAYLOAD - 4 || (int64_t)len > PBC_MAX_PAYLOAD) return -1; /* :226-230 */
  put_be(out, 4, (uint64_t)len + 4);                                                  /* :233 */
  memcpy(out + 4, payload, len);                                                       /* :234 */
  put_be(out + 4 + len, 4, oracle_crc32_long(payload, len));                          /* :238-247 */
  *out_len = 4 + len + 4;
  return 1;
}

/* ProtobufCodec::decode (:127-173) on `size` readable bytes; as oracle_lhc_decode. */
int oracle_pbc_decode(const unsigned char* s, size_t size, size_t* payload_off, size_t* payload_len,
                      size_t* consumed) {
  *payload_off = *payload_len = *consumed = 0;
  if (size < 4) return 0;                                                      /* :150 */
  const int64_t length = (int32_t)(((uint32_t)s[0] << 24) | ((uint32_t)s[1] << 16) | ((uint32_t)s[2] << 8) | s[3]);
  if (length < PBC_MIN_PAYLOAD || length > PBC_MAX_PAYLOAD) return -1;         /* :152-156 */
  if (size - 4 < (uint64_t)length) return 0;                                   /* :157 */
  const unsigned char* tr = s + 4 + length - 4;
  uint32_t want = ((uint32_t)tr[0] << 24) | ((uint32_t)tr[1] << 16) | ((uint32_t)tr[2] << 8) | tr[3];
  if (oracle_crc32_long(s + 4, (size_t)length - 4) != want) return -1;         /* :159-173 */
  *payload_off = 4;
  *payload_len = (size_t)length - 4;
  *consumed = 4 + (size_t)length;
  return 1;
}
