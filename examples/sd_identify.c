/*
 * sd_identify.c — the file-identifier hot path driven through the C ABI alone, the way a
 * compiled host (the Rust core) embeds libsd_hip_cas.so: no Python, no
 * torch, one HIP runtime (/opt/rocm's) in the process.
 *
 *   sd_identify <dir> [chunk] [data_dir] [library_id]
 *
 * 1. walks <dir> (regular files, sorted by path = the file_path id order of a fresh
 *    library) and takes fs::metadata().len() of each (file_identifier/mod.rs:63,78-79);
 *    the job's orphan query skips file_paths indexed with size 0
 *    (orphan_path_filters, file_identifier_job.rs:264), so empty files are reported but
 *    are not rows of the job;
 * 2. one batched generate_cas_id over all of them (sd_cas_generate_cas_ids_from_paths —
 *    cas.rs:23-62 with the reference's reads/seeks; per-file errno like mod.rs:125-141);
 * 3. the Object decisions of the whole identifier job, `chunk` rows per step with the
 *    reference's cursor (sd_cas_identifier_links — file_identifier_job.rs:180-319,
 *    mod.rs:98-350);
 * 4. the thumbnail path of every hashed file (sd_cas_thumbnail_path — thumbnail/mod.rs:67-82)
 *    when data_dir is given (library_id omitted = ephemeral).
 * Prints one JSON object per file, then one per job step.  Exit status 0 on success.
 */
#define _XOPEN_SOURCE 700
#include <errno.h>
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
  return strcmp(g_paths[*(const size_t*)a], g_paths[*(const size_t*)b]);
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
    fprintf(stderr, "usage: %s <dir> [chunk] [data_dir] [library_id]\n", argv[0]);
    return 2;
  }
  const uint32_t chunk = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : SD_CAS_CHUNK_SIZE;
  const char* data_dir = argc > 3 ? argv[3] : NULL;
  const char* library = argc > 4 ? argv[4] : NULL;
  if (nftw(argv[1], visit, 64, FTW_PHYS) != 0) {
    fprintf(stderr, "walk %s: %s\n", argv[1], strerror(errno));
    return 1;
  }
  /* ascending path order */
  size_t* ord = malloc((g_n ? g_n : 1) * sizeof *ord);
  for (size_t i = 0; i < g_n; i++) ord[i] = i;
  qsort(ord, g_n, sizeof *ord, by_path);
  const char** paths = malloc((g_n ? g_n : 1) * sizeof *paths);
  uint64_t* sizes = malloc((g_n ? g_n : 1) * 8);
  for (size_t i = 0; i < g_n; i++) {
    paths[i] = g_paths[ord[i]];
    sizes[i] = g_sizes[ord[i]];
  }
  sd_cas_ctx* ctx = NULL;
  int rc = sd_cas_ctx_create(0, &ctx);
  if (rc != SD_CAS_OK) {
    fprintf(stderr, "sd_cas_ctx_create: %d (%s)\n", rc, sd_cas_last_error(NULL));
    return 1;
  }
  /* the job's rows: the non-empty files (orphan_path_filters), in id order */
  const size_t n = g_n;
  size_t m = 0;
  const char** hp = malloc((n ? n : 1) * sizeof *hp);
  uint64_t* hs = malloc((n ? n : 1) * 8);
  for (size_t i = 0; i < n; i++)
    if (sizes[i] != 0) {
      hp[m] = paths[i];
      hs[m++] = sizes[i];
    }
  uint64_t* keys = calloc(m ? m : 1, 8);
  int32_t* status = calloc(m ? m : 1, 4);
  uint8_t* state = calloc(m ? m : 1, 1);
  /* FileMetadata::new per row (mod.rs:55-95) behind the ABI: sizes NULL = the library takes
   * fs::metadata itself (the walk's sizes are the indexer's, only used for the orphan filter) */
  if (m && (rc = sd_cas_generate_cas_ids_from_paths(ctx, hp, NULL, m, keys, status)) != SD_CAS_OK) {
    fprintf(stderr, "generate_cas_ids_from_paths: %d (%s)\n", rc, sd_cas_last_error(ctx));
    return 1;
  }
  /* a row whose length is 0 by now has no cas_id (mod.rs:78-86); a failed metadata/read is
   * an ERROR row (dropped from its step, mod.rs:125-141) */
  for (size_t j = 0; j < m; j++)
    state[j] = status[j] == SD_CAS_STATUS_NO_CAS ? SD_CAS_ROW_NO_CAS
               : status[j] ? SD_CAS_ROW_ERROR : SD_CAS_ROW_HASHED;
  const size_t max_steps = sd_cas_identifier_max_steps(m, chunk);
  uint32_t* step = calloc(m ? m : 1, 4);
  uint32_t* object = calloc(m ? m : 1, 4);
  uint8_t* action = calloc(m ? m : 1, 1);
  uint64_t* counts = calloc(2 * (max_steps ? max_steps : 1), 8);
  uint64_t steps = 0;
  if ((rc = sd_cas_identifier_links(ctx, keys, state, m, chunk, step, object, action, counts,
                                    max_steps, &steps)) != SD_CAS_OK) {
    fprintf(stderr, "identifier_links: %d (%s)\n", rc, sd_cas_last_error(ctx));
    return 1;
  }
  static const char* act[] = {"created", "linked", "dropped", "not_reached"};
  for (size_t i = 0, j = 0; i < n; i++) {
    printf("{\"path\": ");
    json_str(paths[i]);
    printf(", \"size\": %llu", (unsigned long long)sizes[i]);
    if (sizes[i] == 0) {  /* not an orphan row of the job */
      printf(", \"row\": null, \"cas_id\": null, \"action\": \"not_queried\"}\n");
      continue;
    }
    printf(", \"row\": %zu", j);
    if (state[j] == SD_CAS_ROW_HASHED) {
      char hex[17];
      sd_cas_key_to_hex(keys[j], hex);
      printf(", \"cas_id\": \"%s\"", hex);
      if (data_dir) {
        char tp[4096];
        if (sd_cas_thumbnail_path(data_dir, library, keys[j], tp, sizeof tp) < (int64_t)sizeof tp) {
          printf(", \"thumbnail\": ");
          json_str(tp);
        }
      }
    } else {
      printf(", \"cas_id\": null");
    }
    printf(", \"errno\": %d", status[j] < 0 ? -status[j] : 0);
    if (step[j] == SD_CAS_NO_STEP) printf(", \"step\": null");
    else printf(", \"step\": %u", step[j]);
    if (object[j] == SD_CAS_NO_OBJECT) printf(", \"object\": null");
    else printf(", \"object\": %u", object[j]);
    printf(", \"action\": \"%s\"}\n", action[j] < 4 ? act[action[j]] : "?");
    j++;
  }
  for (uint64_t k = 0; k < steps; k++)
    printf("{\"step\": %llu, \"total_created\": %llu, \"total_linked\": %llu}\n",
           (unsigned long long)k, (unsigned long long)counts[2 * k],
           (unsigned long long)counts[2 * k + 1]);
  sd_cas_ctx_destroy(ctx);
  return 0;
}
