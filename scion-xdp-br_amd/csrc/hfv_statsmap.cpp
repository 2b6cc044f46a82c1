// hfv_statsmap.cpp -- the pinned verdict-counter map: a file-backed equivalent of the per-CPU
// BPF hash map /sys/fs/bpf/<br>/port_stats_map (br/src/bpf/maps.h, pinned by
// br_loader.cpp:136-140) that `br-loader watch <br> <iface>` reads (br_loader.cpp:162-180,
// stats.cpp:116-144).  The data path adds each batch's hfv_br_process counters to it; any
// number of readers poll it.
//
// File layout (little-endian): 16-byte header {magic "HFVSTAT1", u32 version, u32 0}, then
// u64 counters [HFV_BR_STATS_IFINDEX][bytes, packets][HFV_BR_COUNTERS].  Writers hold an
// exclusive flock and add with 64-bit atomics, so a reader sees every counter whole (the
// per-CPU BPF map gives no cross-counter consistency either).
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "hfv_internal.h"

namespace hfv {

static const size_t kStatsWords = HFV_BR_STATS_IFINDEX * 2 * HFV_BR_COUNTERS;
struct StatsFile {
    char magic[8];
    uint32_t version;
    uint32_t pad;
    uint64_t c[kStatsWords];
};
static const char kStatsMagic[8] = {'H', 'F', 'V', 'S', 'T', 'A', 'T', '1'};

static int mkdir_parents(const char *path)
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

static int open_stats(const char *path, bool write, StatsFile **out)
{
    if (write) {
        int rc = mkdir_parents(path);
        if (rc) return rc;
    }
    int fd = open(path, write ? O_RDWR | O_CREAT : O_RDONLY, 0644);
    if (fd < 0) return -errno;
    if (write && flock(fd, LOCK_EX) != 0) { int e = -errno; close(fd); return e; }
    struct stat st;
    if (fstat(fd, &st) != 0) { int e = -errno; close(fd); return e; }
    if (st.st_size == 0 && write) {
        if (ftruncate(fd, sizeof(StatsFile)) != 0) { int e = -errno; close(fd); return e; }
    } else if ((size_t)st.st_size != sizeof(StatsFile)) {
        close(fd);
        return -EINVAL;
    }
    void *m = mmap(nullptr, sizeof(StatsFile), write ? PROT_READ | PROT_WRITE : PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { int e = -errno; close(fd); return e; }
    StatsFile *sf = (StatsFile *)m;
    if (memcmp(sf->magic, kStatsMagic, 8) != 0) {
        if (!write || sf->magic[0] != 0) { munmap(m, sizeof(StatsFile)); close(fd); return -EINVAL; }
        memcpy(sf->magic, kStatsMagic, 8);
        sf->version = 1;
    }
    *out = sf;
    return fd;
}

}  // namespace hfv

using namespace hfv;

extern "C" {

int hfv_statsmap_path(const char *br, char *out, size_t len)
{
    if (!br || !out || !*br || strchr(br, '/')) return fail(-EINVAL, "invalid BR name");
    const char *base = getenv("HFV_PIN_DIR");
    if (!base || !*base) base = "/dev/shm/hfv";
    int w = snprintf(out, len, "%s/%s/port_stats_map", base, br);
    if (w < 0 || (size_t)w >= len) return fail(-ENAMETOOLONG, "path too long");
    return 0;
}

int hfv_statsmap_add(const char *path, const uint64_t *stats)
{
    if (!path || !stats) return fail(-EINVAL, "null argument");
    StatsFile *sf;
    int fd = open_stats(path, true, &sf);
    if (fd < 0) return fail(fd, "cannot open stats map %s", path);
    for (size_t k = 0; k < kStatsWords; ++k)
        if (stats[k]) __atomic_fetch_add(&sf->c[k], stats[k], __ATOMIC_RELAXED);
    munmap(sf, sizeof(StatsFile));
    close(fd);
    return 0;
}

int hfv_statsmap_read(const char *path, uint64_t *stats)
{
    if (!path || !stats) return fail(-EINVAL, "null argument");
    StatsFile *sf;
    int fd = open_stats(path, false, &sf);
    if (fd < 0) return fail(fd, "cannot open stats map %s", path);
    for (size_t k = 0; k < kStatsWords; ++k) stats[k] = __atomic_load_n(&sf->c[k], __ATOMIC_RELAXED);
    munmap(sf, sizeof(StatsFile));
    close(fd);
    return 0;
}

}  // extern "C"
