// Context-adaptive binary range coder for the quantized latent codes (host code).
//
// Replaces the reference's CABAC stage, cabac_compression.py:60-406 (ContextModel, ArithmeticCoder,
// cabac_encode / cabac_decode), which cannot run: its encoder overflows the byte range at :197 after
// _handle_underflow (:210) lets `high` exceed 32 bits.  Same job, same context idea:
//   * symbols are the codebook indices [N, num_ws, w_dim] (< 2^nbits, nbits <= 8);
//   * each symbol is binarised along a bit tree (MSB first), every tree node an adaptive binary probability
//     (11-bit, shift-5 update), coded by a carry-propagating range coder (32-bit range, byte output);
//   * the context of a symbol is the reference's pair (:78-117): the previous symbol in the same w vector
//     and the symbol at the same position of the previous w vector, each bucketed to its top two bits
//     (or "none" at a border) -> 25 bit trees per stream.
// Entropy coding is sequential, so it runs on the host: one independent stream per image (the batch
// dimension), streams coded in parallel on std::threads.  Deterministic: the bytes depend only on the codes.
#include "common.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace ic2 {
namespace {

constexpr int kProbBits = 11, kProbInit = 1 << (kProbBits - 1), kMove = 5;
constexpr uint32_t kTop = 1u << 24;
constexpr int kCtx = 25;

struct RcEncoder {
  uint64_t low = 0;
  uint32_t range = 0xFFFFFFFFu;
  uint8_t cache = 0;
  uint64_t cache_size = 1;
  std::vector<uint8_t>& out;
  explicit RcEncoder(std::vector<uint8_t>& o) : out(o) {}
  void shift_low() {
    if ((uint32_t)low < 0xFF000000u || (low >> 32) != 0) {
      const uint8_t carry = (uint8_t)(low >> 32);
      uint8_t t = cache;
      do {
        out.push_back((uint8_t)(t + carry));
        t = 0xFF;
      } while (--cache_size != 0);
      cache = (uint8_t)(low >> 24);
    }
    ++cache_size;
    low = (low & 0x00FFFFFFu) << 8;
  }
  void bit(uint16_t& p, int b) {
    const uint32_t bound = (range >> kProbBits) * p;
    if (b == 0) {
      range = bound;
      p = (uint16_t)(p + (((1 << kProbBits) - p) >> kMove));
    } else {
      low += bound;
      range -= bound;
      p = (uint16_t)(p - (p >> kMove));
    }
    while (range < kTop) {
      range <<= 8;
      shift_low();
    }
  }
  void flush() {
    for (int i = 0; i < 5; ++i) shift_low();
  }
};

struct RcDecoder {
  const uint8_t* in;
  int64_t n, pos = 0;
  uint32_t range = 0xFFFFFFFFu, code = 0;
  RcDecoder(const uint8_t* p, int64_t len) : in(p), n(len) {
    for (int i = 0; i < 5; ++i) code = (code << 8) | next();
  }
  uint8_t next() { return pos < n ? in[pos++] : 0; }
  int bit(uint16_t& p) {
    const uint32_t bound = (range >> kProbBits) * p;
    int b;
    if (code < bound) {
      range = bound;
      p = (uint16_t)(p + (((1 << kProbBits) - p) >> kMove));
      b = 0;
    } else {
      code -= bound;
      range -= bound;
      p = (uint16_t)(p - (p >> kMove));
      b = 1;
    }
    while (range < kTop) {
      range <<= 8;
      code = (code << 8) | next();
    }
    return b;
  }
};

struct Model {
  int nbits;
  std::vector<uint16_t> p;  // [kCtx][256] bit-tree nodes (index 1 .. 2^nbits - 1)
  explicit Model(int nb) : nbits(nb), p((size_t)kCtx * 256, (uint16_t)kProbInit) {}
  int bucket(int v) const { return v < 0 ? 0 : 1 + (v >> (nbits - 2 > 0 ? nbits - 2 : 0)); }
  uint16_t* tree(int prev_dim, int prev_ws) { return p.data() + (size_t)(bucket(prev_dim) * 5 + bucket(prev_ws)) * 256; }
};

int nbits_for(int n_symbols) {
  int b = 1;
  while ((1 << b) < n_symbols) ++b;
  return b < 2 ? 2 : b;
}

void encode_stream(const int32_t* c, int num_ws, int w_dim, int nbits, std::vector<uint8_t>& out) {
  RcEncoder enc(out);
  Model m(nbits);
  for (int ws = 0; ws < num_ws; ++ws)
    for (int d = 0; d < w_dim; ++d) {
      const int sym = c[ws * w_dim + d];
      uint16_t* t = m.tree(d > 0 ? c[ws * w_dim + d - 1] : -1, ws > 0 ? c[(ws - 1) * w_dim + d] : -1);
      int node = 1;
      for (int i = nbits - 1; i >= 0; --i) {
        const int b = (sym >> i) & 1;
        enc.bit(t[node], b);
        node = (node << 1) | b;
      }
    }
  enc.flush();
}

void decode_stream(const uint8_t* in, int64_t len, int num_ws, int w_dim, int nbits, int32_t* c) {
  RcDecoder dec(in, len);
  Model m(nbits);
  for (int ws = 0; ws < num_ws; ++ws)
    for (int d = 0; d < w_dim; ++d) {
      uint16_t* t = m.tree(d > 0 ? c[ws * w_dim + d - 1] : -1, ws > 0 ? c[(ws - 1) * w_dim + d] : -1);
      int node = 1;
      for (int i = 0; i < nbits; ++i) node = (node << 1) | dec.bit(t[node]);
      c[ws * w_dim + d] = node - (1 << nbits);
    }
}

template <typename F>
void parallel_for(int64_t n, int n_threads, F&& f) {
  int th = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  th = std::max(1, std::min<int>(th, 16));
  th = (int)std::min<int64_t>(th, n);
  if (th <= 1) {
    for (int64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < th; ++t)
    pool.emplace_back([&, t] {
      for (int64_t i = t; i < n; i += th) f(i);
    });
  for (auto& p : pool) p.join();
}

}  // namespace
}  // namespace ic2

using namespace ic2;

extern "C" int64_t ic2_rc_bound(int64_t n_streams, int64_t per_stream) {
  // <= 6.05 bits per binary decision at the probability floor (31/2048), 8 decisions per symbol
  return n_streams * (per_stream * 7 + 16);
}

extern "C" int ic2_rc_encode(const int32_t* codes, int64_t n_streams, int num_ws, int w_dim, int n_symbols,
                             uint8_t* out, int64_t out_cap, int64_t* stream_bytes, int n_threads) {
  IC2_CHECK_ARG(codes && out && stream_bytes && n_streams > 0 && num_ws > 0 && w_dim > 0, "rc_encode: bad arguments");
  IC2_CHECK_ARG(n_symbols >= 2 && n_symbols <= 256, "rc_encode: n_symbols must be in [2, 256], got %d", n_symbols);
  const int64_t per = (int64_t)num_ws * w_dim;
  for (int64_t i = 0; i < n_streams * per; ++i)
    IC2_CHECK_ARG(codes[i] >= 0 && codes[i] < n_symbols, "rc_encode: code %d at %lld outside [0, %d)", codes[i],
                  (long long)i, n_symbols);
  const int nbits = nbits_for(n_symbols);
  std::vector<std::vector<uint8_t>> bufs((size_t)n_streams);
  parallel_for(n_streams, n_threads, [&](int64_t s) {
    bufs[(size_t)s].reserve((size_t)per * 2);
    encode_stream(codes + s * per, num_ws, w_dim, nbits, bufs[(size_t)s]);
  });
  int64_t total = 0;
  for (auto& b : bufs) total += (int64_t)b.size();
  IC2_CHECK_ARG(total <= out_cap, "rc_encode: output capacity %lld < %lld bytes", (long long)out_cap,
                (long long)total);
  int64_t off = 0;
  for (int64_t s = 0; s < n_streams; ++s) {
    std::memcpy(out + off, bufs[(size_t)s].data(), bufs[(size_t)s].size());
    stream_bytes[s] = (int64_t)bufs[(size_t)s].size();
    off += stream_bytes[s];
  }
  return IC2_OK;
}

extern "C" int ic2_rc_decode(const uint8_t* in, const int64_t* stream_bytes, int64_t n_streams, int num_ws, int w_dim,
                             int n_symbols, int32_t* codes_out, int n_threads) {
  IC2_CHECK_ARG(in && stream_bytes && codes_out && n_streams > 0 && num_ws > 0 && w_dim > 0,
                "rc_decode: bad arguments");
  IC2_CHECK_ARG(n_symbols >= 2 && n_symbols <= 256, "rc_decode: n_symbols must be in [2, 256], got %d", n_symbols);
  std::vector<int64_t> offs((size_t)n_streams + 1, 0);
  for (int64_t s = 0; s < n_streams; ++s) {
    IC2_CHECK_ARG(stream_bytes[s] >= 5, "rc_decode: stream %lld is truncated (%lld bytes)", (long long)s,
                  (long long)stream_bytes[s]);
    offs[(size_t)s + 1] = offs[(size_t)s] + stream_bytes[s];
  }
  const int64_t per = (int64_t)num_ws * w_dim;
  const int nbits = nbits_for(n_symbols);
  parallel_for(n_streams, n_threads, [&](int64_t s) {
    decode_stream(in + offs[(size_t)s], stream_bytes[s], num_ws, w_dim, nbits, codes_out + s * per);
  });
  // a corrupt stream can decode symbols >= n_symbols when n_symbols is not a power of two
  for (int64_t i = 0; i < n_streams * per; ++i)
    IC2_CHECK_ARG(codes_out[i] < n_symbols, "rc_decode: corrupt stream (symbol %d >= %d)", codes_out[i], n_symbols);
  return IC2_OK;
}
