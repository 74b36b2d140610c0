// dkey.h — normalized key record shared by host packing and the gfx950 kernels.
//
// A key (unsigned byte string, memcmp-then-length order: SkipList.cpp:53-60,
// flow/Arena.h:692-697) is held as its first 16 bytes, zero-padded, read as two
// big-endian u64 words (integer order == byte order), its full length, and —
// only when it is longer than 16 bytes — the offset of bytes [16, len) in a
// tail arena.  Exactness: if the padded prefixes tie and either
// key is <= 16 bytes, the shorter key is a prefix of the longer, so comparing
// lengths decides; only when both exceed 16 bytes are the tails compared.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define FDB_HD __host__ __device__ __forceinline__
#else
#define FDB_HD inline
#endif

struct __attribute__((aligned(8))) DKey {
    uint64_t hi, lo;  // big-endian words of the zero-padded 16-byte prefix
    uint32_t len;     // full key length in bytes
    uint32_t tail;    // offset of bytes [16, len) in the owning tail arena (len > 16)
};
static_assert(sizeof(DKey) == 24, "DKey is 24 bytes");

// Sort item: a batch endpoint with its key (KeyInfo, SkipList.cpp:77-87).
// meta = range_id << 3 | is_end << 2 | class, class as extra_ordering
// (SkipList.cpp:89-91): read-end 0 < write-end 1 < write-begin 2 < read-begin 3.
// nx = key bytes [16, 19) as a big-endian 24-bit word, zero past the key's end: with it the sort
// needs the tail arena only when both keys exceed kSortNxLen bytes and agree on 19 (a hot key k and
// its end key k\0 of singleKeyRange(k), C3, never do).  A bitonic padding item has meta kPadMeta
// (no endpoint has is_end = 1 with the read-begin class).
struct __attribute__((aligned(16))) SortItem {
    uint64_t hi, lo;
    uint32_t len, tail;
    uint32_t meta, nx;
};
constexpr uint32_t kSortNxLen = 19;
// nx bit 31 (slab items of k_sort_partition only): the endpoint is the end of a non-empty range
// (its key differs from its begin's), which orders the two ends of one range inside the bucket
// sort without their tails; the 24 key bits below it are what every comparison reads.
constexpr uint32_t kNxEndFlag = 1u << 31;
constexpr uint32_t kPadMeta = 0xffffffffu;
static_assert(sizeof(SortItem) == 32, "SortItem is 32 bytes");

enum PointClass : uint32_t { kReadEnd = 0, kWriteEnd = 1, kWriteBegin = 2, kReadBegin = 3 };

FDB_HD uint32_t item_class(uint32_t meta) { return meta & 3u; }
FDB_HD uint32_t item_range(uint32_t meta) { return meta >> 3; }
FDB_HD uint32_t item_is_end(uint32_t meta) { return (meta >> 2) & 1u; }

#if defined(__HIP_DEVICE_COMPILE__)
// Eight tail bytes starting at p as a big-endian word, from the two aligned words that hold them
// (tail arenas start 8-aligned and carry >= 40 bytes of slack past their last tail, so the
// aligned loads of tail_cmp stay inside the allocation).
__device__ __forceinline__ uint64_t tail_word(const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    const uint64_t* w = (const uint64_t*)(a & ~(uintptr_t)7);
    const uint32_t sh = (uint32_t)(a & 7u) * 8u;
    const uint64_t x = w[0], y = w[1];
    return __builtin_bswap64(sh ? (x >> sh) | (y << (64u - sh)) : x);
}
#endif

// Compare the bytes of two tails [16, min(la, lb)) then lengths.  On the device, 32 bytes per
// step as big-endian words (bytes past the shorter tail masked off): a C4 tuple key shares up to
// ~80 tail bytes with its neighbours, and a byte loop pays one dependent load per byte.
FDB_HD int tail_cmp(const uint8_t* ta, uint32_t la, const uint8_t* tb, uint32_t lb) {
    uint32_t n = (la < lb ? la : lb) - 16u;
#if defined(__HIP_DEVICE_COMPILE__)
    for (uint32_t i = 0; i < n; i += 32) {
        uint64_t a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; j++) a[j] = tail_word(ta + i + 8 * j), b[j] = tail_word(tb + i + 8 * j);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int vb = (int)(n - i) - 8 * j;  // bytes of word j inside the shorter tail
            if (vb <= 0) break;
            const uint64_t msk = vb >= 8 ? ~0ull : ~0ull << (64 - 8 * vb);
            const uint64_t x = a[j] & msk, y = b[j] & msk;
            if (x != y) return x < y ? -1 : 1;
        }
    }
#else
    for (uint32_t i = 0; i < n; i++) {
        uint8_t a = ta[i], b = tb[i];
        if (a != b) return a < b ? -1 : 1;
    }
#endif
    return (la > lb) - (la < lb);
}

// Full key order.  arenaA / arenaB are the tail arenas the two keys index.
FDB_HD int key_cmp(uint64_t ahi, uint64_t alo, uint32_t alen, uint32_t atail, const uint8_t* arenaA,
                   uint64_t bhi, uint64_t blo, uint32_t blen, uint32_t btail, const uint8_t* arenaB) {
    if (ahi != bhi) return ahi < bhi ? -1 : 1;
    if (alo != blo) return alo < blo ? -1 : 1;
    if (alen > 16u && blen > 16u) return tail_cmp(arenaA + atail, alen, arenaB + btail, blen);
    return (alen > blen) - (alen < blen);
}

FDB_HD int dkey_cmp(const DKey& a, const uint8_t* arenaA, const DKey& b, const uint8_t* arenaB) {
    return key_cmp(a.hi, a.lo, a.len, a.tail, arenaA, b.hi, b.lo, b.len, b.tail, arenaB);
}

// KeyInfo::operator< (SkipList.cpp:114-128): key, then class.
FDB_HD bool item_less(const SortItem& a, const SortItem& b, const uint8_t* arena) {
    int c = key_cmp(a.hi, a.lo, a.len, a.tail, arena, b.hi, b.lo, b.len, b.tail, arena);
    if (c) return c < 0;
    return item_class(a.meta) < item_class(b.meta);
}

// Host-side normalization of a key into a DKey (prefix words + length); the caller
// appends bytes [16, len) to its tail arena and fills `tail`.
inline void dkey_prefix(const uint8_t* p, uint32_t len, uint64_t* hi, uint64_t* lo) {
    uint8_t buf[16] = {0};
    for (uint32_t i = 0; i < len && i < 16; i++) buf[i] = p[i];
    uint64_t h = 0, l = 0;
    for (int i = 0; i < 8; i++) h = (h << 8) | buf[i];
    for (int i = 8; i < 16; i++) l = (l << 8) | buf[i];
    *hi = h;
    *lo = l;
}
