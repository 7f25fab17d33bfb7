/*
 * sd_validate.c — the object validator job driven through the C ABI alone (no Python, no
 * torch): every regular file under <dir>, sorted by path (the order of the job's
 * file_path steps), gets the full-content BLAKE3 checksum of file_checksum
 * (core/src/object/validation/hash.rs:11-25) from ONE sd_cas_file_checksums call instead
 * of one job step per file (validator_job.rs:107-172).
 *
 *   sd_validate <dir>
 *
 * Prints one JSON object per file: {"path", "size", "integrity_checksum" | null, "errno"}.
 * A file whose read fails gets errno (the reference's step fails with FileIOError,
 * validator_job.rs:149-151).  Exit status 0 on success.
 */
#define _XOPEN_SOURCE 700
#include <ftw.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "sd_hip_cas.h"

static char** g_paths;
static uint64_t* g_sizes;
static size_t g_n, g_cap;

static int visit(const char* p, const struct stat* st, int type, struct FTW* f) {
  (void)f;
  if (type != FTW_F || !S_ISREG(st->st_mode)) return 0;
  if (g_n == g_cap) {
    g_cap = g_cap ? 2 * g_cap : 1024;
    g_paths = realloc(g_paths, g_cap * sizeof *g_paths);
    g_sizes = realloc(g_sizes, g_cap * sizeof *g_sizes);
    if (!g_paths || !g_sizes) return -1;
  }
  g_paths[g_n] = strdup(p);
  g_sizes[g_n] = (uint64_t)st->st_size;
  g_n++;
  return 0;
}

static int by_path(const void* a, const void* b) {
  return strcmp(*(char* const*)a, *(char* const*)b);
}

static void json_str(const char* s) {
  putchar('"');
  for (; *s; s++) {
    if (*s == '"' || *s == '\\') printf("\\%c", *s);
    else if ((unsigned char)*s < 0x20) printf("\\u%04x", (unsigned char)*s);
    else putchar(*s);
  }
  putchar('"');
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s <dir>\n", argv[0]);
    return 2;
  }
  if (nftw(argv[1], visit, 64, FTW_PHYS) != 0) {
    fprintf(stderr, "walk of %s failed\n", argv[1]);
    return 1;
  }
  /* sizes were only needed for the report: re-stat after sorting the paths */
  qsort(g_paths, g_n, sizeof *g_paths, by_path);
  for (size_t i = 0; i < g_n; i++) {
    struct stat st;
    g_sizes[i] = stat(g_paths[i], &st) == 0 ? (uint64_t)st.st_size : 0;
  }
  sd_cas_ctx* ctx = NULL;
  int rc = sd_cas_ctx_create(0, &ctx);
  if (rc != SD_CAS_OK) {
    fprintf(stderr, "sd_cas_ctx_create: %d (%s)\n", rc, sd_cas_last_error(NULL));
    return 1;
  }
  char* hex = malloc(65 * (g_n ? g_n : 1));
  int32_t* status = malloc(sizeof(int32_t) * (g_n ? g_n : 1));
  if (!hex || !status) return 1;
  rc = sd_cas_file_checksums(ctx, (const char* const*)g_paths, g_n, hex, status);
  if (rc != SD_CAS_OK) {
    fprintf(stderr, "sd_cas_file_checksums: %d (%s)\n", rc, sd_cas_last_error(ctx));
    sd_cas_ctx_destroy(ctx);
    return 1;
  }
  for (size_t i = 0; i < g_n; i++) {
    printf("{\"path\": ");
    json_str(g_paths[i]);
    printf(", \"size\": %llu, \"integrity_checksum\": ", (unsigned long long)g_sizes[i]);
    if (status[i]) printf("null");
    else printf("\"%s\"", hex + 65 * i);
    printf(", \"errno\": %d}\n", status[i] ? -status[i] : 0);
  }
  sd_cas_ctx_destroy(ctx);
  for (size_t i = 0; i < g_n; i++) free(g_paths[i]);
  free(g_paths);
  free(g_sizes);
  free(hex);
  free(status);
  return 0;
}
