// hfv_keymap.cpp -- the pinned key map: a file-backed equivalent of the BPF hash map
// /sys/fs/bpf/<br>/mac_key_map (br/src/bpf/maps.h:60-67) that `br-loader key add|remove`
// writes from another process (br_loader.cpp:182-261) while the data plane keeps running.
//
// File layout (little-endian): a 64-byte header {magic "HFVKMAP1", u32 version, u32 seq,
// u32 valid[8], 16 B reserved} followed by HFV_MAX_KEYS struct hop_key slots.  Writers take
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

#include "hfv_internal.h"

namespace hfv {

struct KeymapFile {
    char magic[8];
    uint32_t version;
    uint32_t seq;
    uint32_t valid[8];
    uint8_t reserved[16];
    hop_key slot[HFV_MAX_KEYS];
};
static_assert(sizeof(KeymapFile) == 64 + HFV_MAX_KEYS * 192, "keymap layout");
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

// Open (creating if asked) and map the file; returns the fd, the mapping in *out.
static int map_file(const char *path, bool create, bool writable, KeymapFile **out)
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
        return -EINVAL;
    }
    void *m = mmap(nullptr, sizeof(KeymapFile), writable ? PROT_READ | PROT_WRITE : PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { int e = -errno; close(fd); return e; }
    KeymapFile *km = (KeymapFile *)m;
    if (writable && memcmp(km->magic, kMagic, 8) != 0) {
        if (st.st_size != 0 && km->magic[0] != 0) { munmap(m, sizeof(KeymapFile)); close(fd); return -EINVAL; }
        memcpy(km->magic, kMagic, 8);
        km->version = 1;
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

int keymap_create(const char *path)
{
    KeymapFile *km;
    int fd = map_file(path, true, true, &km);   // header written under the flock, slots untouched
    if (fd < 0) return fd;
    unmap_file(fd, km);
    return 0;
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
    if (index >= HFV_MAX_KEYS) return fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    KeymapFile *km;
    int fd = map_file(path, true, true, &km);
    if (fd < 0) return fail(fd, "cannot open key map %s", path);
    seq_begin(km);   // odd: update in progress
    km->slot[index] = *hk;
    km->valid[index >> 5] |= 1u << (index & 31);
    seq_end(km);     // even: published
    unmap_file(fd, km);
    return 0;
}

int hfv_keymap_erase(const char *path, uint32_t index)
{
    if (!path) return fail(-EINVAL, "null argument");
    if (index >= HFV_MAX_KEYS) return fail(-EINVAL, "key index %u >= %d", index, HFV_MAX_KEYS);
    KeymapFile *km;
    int fd = map_file(path, false, true, &km);
    if (fd < 0) return fail(fd, "cannot open key map %s", path);
    int rc = 0;
    if (!((km->valid[index >> 5] >> (index & 31)) & 1u)) {
        rc = fail(-ENOENT, "key slot %u is empty", index);
    } else {
        seq_begin(km);
        km->valid[index >> 5] &= ~(1u << (index & 31));
        memset(&km->slot[index], 0, sizeof(hop_key));
        seq_end(km);
    }
    unmap_file(fd, km);
    return rc;
}

int hfv_keymap_create(const char *path)
{
    if (!path) return fail(-EINVAL, "null argument");
    int rc = keymap_create(path);
    return rc ? fail(rc, "cannot create key map %s", path) : 0;
}

int hfv_keymap_read(const char *path, struct hop_key *slots, uint32_t *valid)
{
    if (!path || !slots || !valid) return fail(-EINVAL, "null argument");
    const void *m;
    int rc = keymap_open_ro(path, &m);
    if (rc) return fail(rc, "cannot open key map %s", path);
    keymap_snapshot(m, slots, valid);
    keymap_close(m);
    return 0;
}

}  // extern "C"
