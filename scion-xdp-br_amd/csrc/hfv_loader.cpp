// hfv-loader -- control-plane CLI for the MI355X hop-field verifier, the counterpart of the
// reference's `br-loader key add|remove` (br/src/br_loader.cpp:50-61, 182-295).
//
//   hfv-loader key add <br> <index> <base64-key>    decode, expand, derive K1, update map
//   hfv-loader key remove <br> <index>              erase the slot (it then fails closed)
//   hfv-loader key list <br>                        print occupied slots and K1 of each
//
// The pinned map lives at $HFV_PIN_DIR/<br>/mac_key_map (default /dev/shm/hfv); a data plane
// that called hfv_ctx_attach_keymap() on it picks the change up at its next batch.  Messages
// and exit codes follow br-loader: errors on stderr, EXIT_FAILURE.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <stdexcept>
#include <string>

#include "../../include/scion_hfv.h"

static void print_usage()
{
    fprintf(stderr,
            "Usage: hfv-loader key add <br> <index> <key>\n"
            "                  key remove <br> <index>\n"
            "                  key list <br>\n");
}

static bool parse_index(const char *s, uint32_t *out)
{
    try {
        size_t pos = 0;
        unsigned long v = std::stoul(std::string(s), &pos);
        if (pos != strlen(s) || v > 0xffffffffUL) return false;
        *out = (uint32_t)v;
        return true;
    } catch (const std::exception &) {
        return false;
    }
}

static int map_path(const char *br, char *path, size_t len)
{
    if (hfv_keymap_path(br, path, len) != 0) {
        fprintf(stderr, "Invalid border router name: %s\n", hfv_last_error());
        return -1;
    }
    return 0;
}

static int add_key(int argc, char **argv)
{
    if (argc < 3) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    uint32_t index;
    if (!parse_index(argv[1], &index)) {
        fprintf(stderr, "Invalid verification key index\n");
        return EXIT_FAILURE;
    }
    struct aes_key key;
    if (hfv_decode_key_b64(argv[2], &key) != 0) {
        fprintf(stderr, "Invalid MAC verification key: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    // the same derivation as br_loader.cpp:213-218: expansion, subkeys, keep K1
    struct hop_key hk;
    aes_key_expansion(&key, &hk.key);
    struct aes_block subkeys[2];
    aes_cmac_subkeys(&hk.key, subkeys);
    hk.subkey = subkeys[0];
    if (hfv_keymap_update(path, index, &hk) != 0) {
        fprintf(stderr, "Update failed: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}

static int remove_key(int argc, char **argv)
{
    if (argc < 2) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    uint32_t index;
    if (!parse_index(argv[1], &index)) {
        fprintf(stderr, "Invalid verification key index\n");
        return EXIT_FAILURE;
    }
    if (hfv_keymap_erase(path, index) != 0) {
        fprintf(stderr, "Update failed: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    return EXIT_SUCCESS;
}

static int list_keys(int argc, char **argv)
{
    if (argc < 1) { print_usage(); return EXIT_FAILURE; }
    char path[4096];
    if (map_path(argv[0], path, sizeof path)) return EXIT_FAILURE;
    static struct hop_key slots[HFV_MAX_KEYS];
    uint32_t valid[8];
    if (hfv_keymap_read(path, slots, valid) != 0) {
        fprintf(stderr, "Cannot read key map: %s\n", hfv_last_error());
        return EXIT_FAILURE;
    }
    for (uint32_t k = 0; k < HFV_MAX_KEYS; ++k) {
        if (!((valid[k >> 5] >> (k & 31)) & 1u)) continue;
        printf("%u K1=", k);
        for (int i = 0; i < 16; ++i) printf("%02x", slots[k].subkey.b[i]);
        printf("\n");
    }
    return EXIT_SUCCESS;
}

int main(int argc, char **argv)
{
    if (argc >= 3 && strcmp(argv[1], "key") == 0) {
        if (strcmp(argv[2], "add") == 0) return add_key(argc - 3, argv + 3);
        if (strcmp(argv[2], "remove") == 0) return remove_key(argc - 3, argv + 3);
        if (strcmp(argv[2], "list") == 0) return list_keys(argc - 3, argv + 3);
    }
    print_usage();
    return EXIT_FAILURE;
}
