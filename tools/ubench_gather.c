// Config-1 gather microbenchmark (host only): the per-file syscall pattern of
// sd_cas_generate_cas_ids_from_paths' gather — open + fstat + the cas.rs:27-58 preads
// (whole file, or header+sample0, samples 1-3, footer) + close — over a file list, on T
// threads pulling files from an atomic cursor; and, where the kernel allows it, the same
// reads submitted through io_uring (one ring per thread, a file's reads as one batch).
// Usage: ubench_gather <list: "path size" lines> <threads> [uring]
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <linux/io_uring.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#define MAXF 200000
static char (*paths)[128];
static uint64_t* sizes;
static int n, use_uring;
static atomic_int next;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

struct ring {
  int fd;
  unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
  struct io_uring_sqe* sqes;
  struct io_uring_cqe* cqes;
};

static int ring_init(struct ring* r, unsigned entries) {
  struct io_uring_params p;
  memset(&p, 0, sizeof p);
  r->fd = (int)syscall(__NR_io_uring_setup, entries, &p);
  if (r->fd < 0) return -errno;
  size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
  size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(struct io_uring_cqe);
  char* sq = mmap(0, sq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_SQ_RING);
  char* cq = mmap(0, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_CQ_RING);
  r->sqes = mmap(0, p.sq_entries * sizeof(struct io_uring_sqe), PROT_READ | PROT_WRITE,
                 MAP_SHARED | MAP_POPULATE, r->fd, IORING_OFF_SQES);
  if (sq == MAP_FAILED || cq == MAP_FAILED || r->sqes == MAP_FAILED) return -ENOMEM;
  r->sq_head = (unsigned*)(sq + p.sq_off.head); r->sq_tail = (unsigned*)(sq + p.sq_off.tail);
  r->sq_mask = (unsigned*)(sq + p.sq_off.ring_mask); r->sq_array = (unsigned*)(sq + p.sq_off.array);
  r->cq_head = (unsigned*)(cq + p.cq_off.head); r->cq_tail = (unsigned*)(cq + p.cq_off.tail);
  r->cq_mask = (unsigned*)(cq + p.cq_off.ring_mask); r->cqes = (struct io_uring_cqe*)(cq + p.cq_off.cqes);
  return 0;
}

static void ring_read(struct ring* r, int fd, void* buf, unsigned len, uint64_t off) {
  unsigned tail = *r->sq_tail, idx = tail & *r->sq_mask;
  struct io_uring_sqe* e = &r->sqes[idx];
  memset(e, 0, sizeof *e);
  e->opcode = IORING_OP_READ; e->fd = fd; e->addr = (uint64_t)(uintptr_t)buf; e->len = len; e->off = off;
  r->sq_array[idx] = idx;
  __atomic_store_n(r->sq_tail, tail + 1, __ATOMIC_RELEASE);
}

static int ring_submit_wait(struct ring* r, unsigned k) {
  if (syscall(__NR_io_uring_enter, r->fd, k, k, IORING_ENTER_GETEVENTS, NULL, 0) < 0) return -errno;
  unsigned head = *r->cq_head;
  while (head != __atomic_load_n(r->cq_tail, __ATOMIC_ACQUIRE)) head++;
  __atomic_store_n(r->cq_head, head, __ATOMIC_RELEASE);
  return 0;
}

static void* work(void* a) {
  (void)a;
  char* buf = aligned_alloc(4096, 128 << 10);
  struct ring r;
  if (use_uring && ring_init(&r, 8) != 0) { fprintf(stderr, "io_uring unavailable\n"); exit(3); }
  for (int i; (i = atomic_fetch_add(&next, 1)) < n;) {
    int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) continue;
    const uint64_t s = sizes[i];
    if (s <= 102400) {
      if (use_uring) { ring_read(&r, fd, buf, (unsigned)s, 0); ring_submit_wait(&r, 1); }
      else if (pread(fd, buf, s, 0) < 0) perror("pread");
    } else {
      const uint64_t j = (s - 16384) / 4;
      if (use_uring) {
        ring_read(&r, fd, buf, 18432, 0);
        for (int k = 1; k < 4; k++) ring_read(&r, fd, buf + 18432 + 10240 * (k - 1), 10240, 8192 + k * j);
        ring_read(&r, fd, buf + 49152, 8192, (uint64_t)st.st_size - 8192);
        ring_submit_wait(&r, 5);
      } else {
        ssize_t x = pread(fd, buf, 18432, 0);
        for (int k = 1; k < 4; k++) x += pread(fd, buf, 10240, 8192 + k * j);
        x += pread(fd, buf, 8192, (off_t)st.st_size - 8192);
        if (x < 0) perror("pread");
      }
    }
    close(fd);
  }
  free(buf);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s list threads [uring]\n", argv[0]); return 2; }
  paths = malloc(sizeof(*paths) * MAXF);
  sizes = malloc(sizeof(*sizes) * MAXF);
  FILE* f = fopen(argv[1], "r");
  if (!f) { perror(argv[1]); return 2; }
  while (n < MAXF && fscanf(f, "%127s %lu", paths[n], &sizes[n]) == 2) n++;
  const int T = atoi(argv[2]);
  use_uring = argc > 3;
  for (int rep = 0; rep < 3; rep++) {
    atomic_store(&next, 0);
    pthread_t th[256];
    const double t = now();
    for (int k = 0; k < T; k++) pthread_create(&th[k], 0, work, 0);
    for (int k = 0; k < T; k++) pthread_join(th[k], 0);
    const double dt = now() - t;
    printf("%s T=%d files=%d %.1f ms %.0f k files/s\n", use_uring ? "uring" : "pread", T, n, dt * 1e3, n / dt / 1e3);
  }
  return 0;
}
