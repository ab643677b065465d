// null_codec.cc -- a TEST DOUBLE of libmemo_ec for profiling the plugin's
// host side on a machine without a GPU (tools/host_profile.sh).  It computes
// nothing: encode and rebuild write zeros, so only the store and healthy
// fetch legs of bench_plugin mean anything with it (MEMO_EC_PLUGIN_HOSTONLY=1
// skips the others).  It is linked into host/_build/hostprof/ only, never
// into the library, the plugin or any test that checks bytes.
#include <cstdlib>
#include <cstring>

#include "../../include/memo_ec.h"

struct memo_ec_ctx {
  int device;
};

extern "C" {
int memo_ec_device_count(void) { return 1; }
int memo_ec_ctx_create(int device, memo_ec_ctx** out) {
  *out = new memo_ec_ctx{device};
  return MEMO_EC_OK;
}
int memo_ec_ctx_destroy(memo_ec_ctx* ctx) {
  delete ctx;
  return MEMO_EC_OK;
}
size_t memo_ec_shard_size(size_t B, int k) {
  if (k < 1) return 0;
  size_t per = (B + (size_t)k - 1) / (size_t)k;
  if (per == 0) per = 1;
  return (per + 63) & ~(size_t)63;
}
int memo_ec_encode_batch(memo_ec_ctx*, int, int m, size_t S, size_t n, const uint8_t*, uint8_t* parity, int) {
  std::memset(parity, 0, (size_t)m * S * n);
  return MEMO_EC_OK;
}
int memo_ec_rebuild_batch(memo_ec_ctx*, int, int, size_t S, size_t n, const uint8_t*, const uint8_t*,
                          const uint8_t*, int e, uint8_t* out, int) {
  std::memset(out, 0, (size_t)e * S * n);
  return MEMO_EC_OK;
}
int memo_ec_rebuild_uniform(memo_ec_ctx*, int, int, size_t S, size_t n, const uint8_t*, const uint8_t*,
                            const uint8_t*, int e, uint8_t* out, int) {
  std::memset(out, 0, (size_t)e * S * n);
  return MEMO_EC_OK;
}
int memo_ec_rebuild_segments(memo_ec_ctx*, int nseg, const memo_ec_rebuild_segment* segs, int) {
  for (int i = 0; i < nseg; ++i) std::memset(segs[i].out, 0, (size_t)segs[i].e * segs[i].S * segs[i].n);
  return MEMO_EC_OK;
}
void* memo_ec_host_alloc(size_t bytes) { return std::malloc(bytes ? bytes : 1); }
int memo_ec_host_free(void* p) {
  std::free(p);
  return MEMO_EC_OK;
}
const char* memo_ec_strerror(int) { return "null codec"; }
}
