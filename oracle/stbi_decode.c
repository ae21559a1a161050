/* TEST INFRASTRUCTURE: decode an image with the reference's vendored stb_image
 * (libs/zstbi/libs/stbi, v2.28) exactly as src/main.zig:1124 does
 * (zstbi.Image.loadFromFile(path, 4) -> forced 4 components) and dump
 * "W H\n" + raw RGBA8 bytes to stdout.  Built into oracle/_ref/ only. */
#include <stdio.h>
#include <stdlib.h>
#include "stb_image.h"
/* zstbi.init (libs/zstbi/src/zstbi.zig:4) installs these allocator hooks */
extern void* (*zstbiMallocPtr)(size_t);
extern void* (*zstbiReallocPtr)(void*, size_t);
extern void (*zstbiFreePtr)(void*);
int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: stbi_decode image\n"); return 2; }
    int w, h, n;
    zstbiMallocPtr = malloc; zstbiReallocPtr = realloc; zstbiFreePtr = free;
    unsigned char* d = stbi_load(argv[1], &w, &h, &n, 4);
    if (!d) { fprintf(stderr, "decode failed\n"); return 1; }
    printf("%d %d\n", w, h);
    fwrite(d, 1, (size_t)w * h * 4, stdout);
    stbi_image_free(d);
    return 0;
}
