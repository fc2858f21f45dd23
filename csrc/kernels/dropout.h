// Counter-based dropout masks shared by the transformer kernels (transformer.hip,
// flash_attn.hip): keep/drop of element i is a hash of (seed, site salt, i), so nothing is
// stored, the backward regenerates the forward's mask, and every kernel that drops the
// same element index drops the same elements (ops/transformer.py keep_mask is the host twin).
#pragma once
#include <cstdint>

static __device__ __forceinline__ uint32_t hash_u32(uint32_t seed, uint32_t salt, uint32_t i) {
  uint32_t x = i * 0x9E3779B9u ^ (seed * 0x85EBCA6Bu + salt * 0xC2B2AE35u);
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// keep with probability 1-p: compare the top 24 bits against the threshold
static __device__ __forceinline__ bool keep(uint32_t seed, uint32_t salt, uint32_t i, uint32_t thr) {
  return (hash_u32(seed, salt, i) >> 8) >= thr;
}
static __host__ __device__ __forceinline__ uint32_t drop_threshold(float p) {
  return (uint32_t)(p * 16777216.0f);
}
