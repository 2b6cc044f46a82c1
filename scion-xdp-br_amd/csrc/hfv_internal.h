// hfv_internal.h -- shared between the host API (hfv_api.cpp, hfv_aes_host.cpp) and the
// kernel launchers (hfv_kernels.hip).  Not installed.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/scion_hfv.h"
#include "hfv_tables.h"

namespace hfv {

// error reporting (thread-local message, negative errno return)
int fail(int code, const char *fmt, ...);

// host AES (hfv_aes_host.cpp)
void expand_key(const uint8_t key[16], uint32_t w[44]);
void encrypt_block(const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]);
void hop_key_from_key(const uint8_t key[16], hop_key *hk);
void compile_dev_key(const hop_key *hk, uint32_t dk[4 * kDevKeyRows]);

// Device key table as the kernels see it: dev keys in round-major order
// [kDevKeyRows][HFV_MAX_KEYS] x 16 B, followed by the 256-bit valid bitmap.
struct DevKeyTable {
    uint32_t rows[kDevKeyRows][HFV_MAX_KEYS][4];
    uint32_t valid[8];
};

enum KernelMode { kModeRecords = 0, kModeMacinputs = 1, kModeTags = 2 };

struct KernelVariant {
    int block;           // threads per block
    int pf;              // record tiles loaded ahead of the one computed (1 or 2)
    int tab;             // round tables in LDS: 2 (T0/T1, 64 KiB) or 4 (T0..T3, 128 KiB)
    int blocks_per_cu;   // persistent grid = num_cus * blocks_per_cu
    int dma;             // 1: fill the LDS tables from ttab_img by LDS-DMA; 0: compute them
    int np;              // packets per lane computed together (1 or 2)
    int dyn;             // 1: waves pull tiles from a per-block LDS queue; 0: static stride
};

struct LaunchGeom {
    int num_cus;
    KernelVariant single;   // KEYSEL_ZERO record verify
    KernelVariant multi;    // KEYSEL_IFID record verify (per-lane keys in LDS)
    const uint32_t *ttab_img;   // 128 KiB device image of the replicated T0..T3 tables
};

// kernel launchers (hfv_kernels.hip); return hipError_t as int
int launch_verify_records(const LaunchGeom &g, const DevKeyTable *tab, int keysel, const uint8_t *recs,
                          size_t stride, size_t n, uint32_t inf_off, uint32_t hf_off, uint64_t *bits,
                          void *stream, void *ev_start = nullptr, void *ev_stop = nullptr);
int launch_verify_macinputs(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint64_t *expected,
                            const uint8_t *kidx, size_t n, uint64_t *bits, void *stream);
int launch_cmac_tags(const LaunchGeom &g, const DevKeyTable *tab, const void *mi, const uint8_t *kidx, size_t n,
                     void *tags, void *stream);
int launch_expand_keys(const uint8_t *raw, size_t n, hop_key *out, DevKeyTable *tab, uint32_t first_slot,
                       void *stream);
int launch_gen_records(const LaunchGeom &g, const DevKeyTable *tab, int keysel, uint8_t *recs, size_t stride,
                       size_t n, uint64_t seed, uint64_t first_index, void *stream);
int query_geometry(int device, LaunchGeom *g);
int launch_verify_stamped(const LaunchGeom &g, const DevKeyTable *tab, const uint8_t *recs, size_t n,
                          uint64_t *bits, uint64_t *stamps, void *stream);
int build_ttab_image(uint32_t *img, void *stream);

// pinned key map (hfv_keymap.cpp)
int keymap_open_ro(const char *path, const void **mapping);
void keymap_close(const void *mapping);
uint32_t keymap_seq(const void *mapping);
uint32_t keymap_snapshot(const void *mapping, hop_key *slots, uint32_t valid[8]);

}  // namespace hfv
