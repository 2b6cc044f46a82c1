// hfv_keymap.cpp -- the pinned key map: a file-backed equivalent of the BPF hash map
// /sys/fs/bpf/<br>/mac_key_map (br/src/bpf/maps.h:60-67) that `br-loader key add|remove`
// writes from another process (br_loader.cpp:182-261) while the data plane keeps running.
//
// File layout (little-endian): a 64-byte header {magic "HFVKMAP1", u32 version, u32 seq,
// u32 valid[8], u32 mode, 12 B reserved} followed by HFV_MAX_KEYS struct hop_key slots and
// kFar entries {u32 index, u32 used, 8 B pad, hop_key} for indices >= HFV_MAX_KEYS.
//
// Two modes, fixed when the map is created:
//   HFV_KEYMAP_SLOTS  256 direct slots, index 0..255 (config 3's per-interface keys);
//   HFV_KEYMAP_HASH8  the reference map's semantics (maps.h:60-67: BPF_MAP_TYPE_HASH, u32 key,
//                     max_entries 8): any u32 index, at most 8 entries -- a 9th new index fails
//                     like bpf_map_update_elem does (E2BIG); indices < 256 live in the direct
//                     slots the data plane reads, larger ones (never looked up: xdp.c:82
//                     reads index 0) in the far entries.
// Writers take
// an exclusive flock and bump `seq` to odd before and to even after the update (a seqlock);
// readers (a ctx attached with hfv_ctx_attach_keymap) poll `seq` once per batch and copy
// the table when it changed, retrying while it is odd or moves underneath them.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <utility>

#include "hfv_internal.h"

namespace hfv {

constexpr int kFar = 8;
struct KeymapFar {
    uint32_t index;
    uint32_t used;
    uint8_t pad[8];
    hop_key key;
};
struct KeymapFile {
    char magic[8];
    uint32_t version;
    uint32_t seq;
    uint32_t valid[8];
    uint32_t mode;   // HFV_KEYMAP_SLOTS (0) or HFV_KEYMAP_HASH8
    uint8_t reserved[12];
    hop_key slot[HFV_MAX_KEYS];
    KeymapFar far[kFar];
};
static_assert(sizeof(KeymapFile) == 64 + HFV_MAX_KEYS * 192 + kFar * 208, "keymap layout");
constexpr uint32_t kHash8Entries = 8;   // maps.h:66 max_entries

static uint32_t entries(const KeymapFile *km)
{
    uint32_t n = 0;
    for (int w = 0; w < 8; ++w) n += (uint32_t)__builtin_popcount(km->valid[w]);
    for (int f = 0; f < kFar; ++f) n += km->far[f].used ? 1u : 0u;
    return n;
}
static const char kMagic[8] = {'H', 'F', 'V', 'K', 'M', 'A', 'P', '1'};

static int mkdir_p(const char *path)
{
    char tmp[4096];
    if (strlen(path) >= sizeof tmp) return -ENAMETOOLONG;
    strcpy(tmp, path);
    for (char *p = tmp + 1; *p; ++p) {
        if (*p != '/') continue;
        *p = 0;
        if (mkdir(tmp, 0755) != 0 && errno != EEXIST) return -errno;
        *p = '/';
    }
    return 0;
}

// Size of a map pinned by the round-2 build, before the far[] entries of HASH8 mode: refused
// with its own error (-EPROTO, "old key map layout") instead of a bare -EINVAL.
constexpr size_t kOldKeymapSize = 64 + HFV_MAX_KEYS * 192;

// Open (creating if asked) and map the file; returns the fd, the mapping in *out; *fresh (if
// given): the file had no map in it yet (created now, or still all zero).
static int map_file(const char *path, bool create, bool writable, KeymapFile **out, bool *fresh = nullptr)
{
    if (create) {
        int rc = mkdir_p(path);
        if (rc) return rc;
    }
    int fd = open(path, (writable ? O_RDWR : O_RDONLY) | (create ? O_CREAT : 0), 0644);
    if (fd < 0) return -errno;
    if (writable && flock(fd, LOCK_EX) != 0) { int e = -errno; close(fd); return e; }
    struct stat st;
    if (fstat(fd, &st) != 0) { int e = -errno; close(fd); return e; }
    if (st.st_size == 0 && create) {
        if (ftruncate(fd, sizeof(KeymapFile)) != 0) { int e = -errno; close(fd); return e; }
    } else if ((size_t)st.st_size != sizeof(KeymapFile)) {
        close(fd);
        return (size_t)st.st_size == kOldKeymapSize ? -EPROTO : -EINVAL;
    }
    void *m = mmap(nullptr, sizeof(KeymapFile), writable ? PROT_READ | PROT_WRITE : PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { int e = -errno; close(fd); return e; }
    KeymapFile *km = (KeymapFile *)m;
    if (fresh) *fresh = false;
    if (writable && memcmp(km->magic, kMagic, 8) != 0) {
        if (st.st_size != 0 && km->magic[0] != 0) { munmap(m, sizeof(KeymapFile)); close(fd); return -EINVAL; }
        memcpy(km->magic, kMagic, 8);
        km->version = 1;
        if (fresh) *fresh = true;
    } else if (!writable && memcmp(km->magic, kMagic, 8) != 0) {
        munmap(m, sizeof(KeymapFile));
        close(fd);
        return -EINVAL;
    }
    *out = km;
    return fd;
}

static void unmap_file(int fd, KeymapFile *km)
{
    msync(km, sizeof(KeymapFile), MS_SYNC);
    munmap(km, sizeof(KeymapFile));
    close(fd);   // releases the flock
}

static inline uint32_t seq_load(const KeymapFile *km)
{
    return __atomic_load_n(&km->seq, __ATOMIC_ACQUIRE);
}

// Seqlock writer side (under the flock).  The odd store must be ordered before the slot
// stores that follow it: a release store alone does not keep later stores behind it, so a
// release fence follows it (a reader that saw the new slot bytes then also sees seq odd).
// The even store is a release store: the slot stores are ordered before it.
static inline void seq_begin(KeymapFile *km)
{
    __atomic_store_n(&km->seq, km->seq + 1, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_release);
}
static inline void seq_end(KeymapFile *km) { __atomic_store_n(&km->seq, km->seq + 1, __ATOMIC_RELEASE); }

// Copy a consistent snapshot; returns the (even) seq it belongs to.
uint32_t keymap_snapshot(const void *mapping, hop_key *slots, uint32_t valid[8])
{
    const KeymapFile *km = (const KeymapFile *)mapping;
    for (;;) {
        uint32_t s0 = seq_load(km);
        if (s0 & 1u) { usleep(10); continue; }
        memcpy(valid, km->valid, 32);
        memcpy(slots, km->slot, sizeof(km->slot));
        std::atomic_thread_fence(std::memory_order_acquire);
        if (seq_load(km) == s0) return s0;
    }
}

uint32_t keymap_seq(const void *mapping) { return seq_load((const KeymapFile *)mapping); }

int keymap_open_ro(const char *path, const void **mapping)
{
    KeymapFile *km;
    int fd = map_file(path, false, false, &km);
    if (fd < 0) return fd;
    close(fd);   // the mapping stays valid
    *mapping = km;
    return 0;
}

void keymap_close(const void *mapping)
{
    if (mapping) munmap((void *)mapping, sizeof(KeymapFile));
}

int keymap_create(const char *path, uint32_t mode)
{
    KeymapFile *km;
    bool fresh = false;
    int fd = map_file(path, true, true, &km, &fresh);   // header written under the flock, slots untouched
    if (fd < 0) return fd;
    // only a map created now takes the mode: an existing one keeps its own, keys or not (an
    // `attach --key-slots` map stays a 256-slot map when `key add` opens it)
    if (fresh) km->mode = mode;
    unmap_file(fd, km);
    return 0;
}

// fail() for a map that could not be opened: an old layout gets its own message.
static int open_fail(int rc, const char *path)
{
    if (rc == -EPROTO)
        return fail(rc, "key map %s has an old layout (%zu bytes, before the HASH8 entries); remove it and add the "
                        "keys again", path, kOldKeymapSize);
    return fail(rc, "cannot open key map %s", path);
}

}  // namespace hfv

using namespace hfv;

extern "C" {

int hfv_keymap_path(const char *br, char *out, size_t len)
{
    if (!br || !out || !*br || strchr(br, '/')) return fail(-EINVAL, "invalid BR name");
    const char *base = getenv("HFV_PIN_DIR");
    if (!base || !*base) base = "/dev/shm/hfv";
    int w = snprintf(out, len, "%s/%s/mac_key_map", base, br);
    if (w < 0 || (size_t)w >= len) return fail(-ENAMETOOLONG, "path too long");
    return 0;
}

int hfv_keymap_update(const char *path, uint32_t index, const struct hop_key *hk)
{
    if (!path || !hk) return fail(-EINVAL, "null argument");
    KeymapFile *km;
    int fd = map_file(path, true, true, &km);   // a map created here is a slots map
    if (fd < 0) return open_fail(fd, path);
    const bool hash8 = km->mode == HFV_KEYMAP_HASH8;
    int far = -1, free_far = -1;
    for (int f = 0; f < kFar; ++f) {
        if (km->far[f].used && km->far[f].index == index) far = f;
        if (!km->far[f].used && free_far < 0) free_far = f;
    }
    const bool exists = index < HFV_MAX_KEYS ? ((km->valid[index >> 5] >> (index & 31)) & 1u) != 0 : far >= 0;
    int rc = 0;
    if (!hash8 && index >= HFV_MAX_KEYS) {
        rc = fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    } else if (hash8 && !exists && entries(km) >= kHash8Entries) {
        rc = fail(-E2BIG, "key map full (%u entries, maps.h:66 max_entries)", kHash8Entries);   // bpf_map_update_elem
    } else {
        seq_begin(km);   // odd: update in progress
        if (index < HFV_MAX_KEYS) {
            km->slot[index] = *hk;
            km->valid[index >> 5] |= 1u << (index & 31);
        } else {
            const int f = far >= 0 ? far : free_far;   // entries < 8 guarantees a free entry
            km->far[f].key = *hk;
            km->far[f].index = index;
            km->far[f].used = 1;
        }
        seq_end(km);     // even: published
    }
    unmap_file(fd, km);
    return rc;
}

int hfv_keymap_erase(const char *path, uint32_t index)
{
    if (!path) return fail(-EINVAL, "null argument");
    KeymapFile *km;
    int fd = map_file(path, false, true, &km);
    if (fd < 0) return open_fail(fd, path);
    int rc = 0, far = -1;
    for (int f = 0; f < kFar; ++f)
        if (km->far[f].used && km->far[f].index == index) far = f;
    if (index >= HFV_MAX_KEYS && km->mode != HFV_KEYMAP_HASH8) {
        rc = fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    } else if (index < HFV_MAX_KEYS ? !((km->valid[index >> 5] >> (index & 31)) & 1u) : far < 0) {
        rc = fail(-ENOENT, "key slot %u is empty", index);
    } else {
        seq_begin(km);
        if (index < HFV_MAX_KEYS) {
            km->valid[index >> 5] &= ~(1u << (index & 31));
            memset(&km->slot[index], 0, sizeof(hop_key));
        } else {
            memset(&km->far[far], 0, sizeof(KeymapFar));
        }
        seq_end(km);
    }
    unmap_file(fd, km);
    return rc;
}

int hfv_keymap_create(const char *path)
{
    if (!path) return fail(-EINVAL, "null argument");
    int rc = keymap_create(path, HFV_KEYMAP_SLOTS);
    return rc == -EPROTO ? open_fail(rc, path) : rc ? fail(rc, "cannot create key map %s", path) : 0;
}

int hfv_keymap_create_mode(const char *path, int mode)
{
    if (!path || (mode != HFV_KEYMAP_SLOTS && mode != HFV_KEYMAP_HASH8)) return fail(-EINVAL, "bad argument");
    int rc = keymap_create(path, (uint32_t)mode);
    return rc == -EPROTO ? open_fail(rc, path) : rc ? fail(rc, "cannot create key map %s", path) : 0;
}

int hfv_keymap_mode(const char *path)
{
    if (!path) return fail(-EINVAL, "null argument");
    const void *m;
    int rc = keymap_open_ro(path, &m);
    if (rc) return open_fail(rc, path);
    const int mode = (int)__atomic_load_n(&((const KeymapFile *)m)->mode, __ATOMIC_ACQUIRE);
    keymap_close(m);
    return mode;
}

int hfv_keymap_list(const char *path, uint32_t *indices, struct hop_key *keys, size_t cap, size_t *count)
{
    if (!path || !count || (cap && (!indices || !keys))) return fail(-EINVAL, "null argument");
    const void *m;
    int rc = keymap_open_ro(path, &m);
    if (rc) return open_fail(rc, path);
    const KeymapFile *km = (const KeymapFile *)m;
    static thread_local KeymapFile snap;
    for (;;) {   // the seqlock reader over the whole file
        const uint32_t s0 = seq_load(km);
        if (s0 & 1u) { usleep(10); continue; }
        memcpy(&snap, km, sizeof snap);
        std::atomic_thread_fence(std::memory_order_acquire);
        if (seq_load(km) == s0) break;
    }
    keymap_close(m);
    size_t n = 0;
    auto put = [&](uint32_t index, const hop_key &k) {
        if (n < cap) {
            indices[n] = index;
            keys[n] = k;
        }
        ++n;
    };
    for (uint32_t i = 0; i < HFV_MAX_KEYS; ++i)
        if ((snap.valid[i >> 5] >> (i & 31)) & 1u) put(i, snap.slot[i]);
    int order[kFar], nf = 0;   // far entries by index
    for (int f = 0; f < kFar; ++f)
        if (snap.far[f].used) order[nf++] = f;
    for (int a = 1; a < nf; ++a)
        for (int b = a; b > 0 && snap.far[order[b]].index < snap.far[order[b - 1]].index; --b) std::swap(order[b], order[b - 1]);
    for (int a = 0; a < nf; ++a) put(snap.far[order[a]].index, snap.far[order[a]].key);
    *count = n;
    return 0;
}

int hfv_keymap_read(const char *path, struct hop_key *slots, uint32_t *valid)
{
    if (!path || !slots || !valid) return fail(-EINVAL, "null argument");
    const void *m;
    int rc = keymap_open_ro(path, &m);
    if (rc) return open_fail(rc, path);
    keymap_snapshot(m, slots, valid);
    keymap_close(m);
    return 0;
}

}  // extern "C"
