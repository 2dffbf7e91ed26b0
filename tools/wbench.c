// Output-file write strategies on the box's file system (host only, no GPU): one writer thread with
// 64 MB pwrites, T threads pwriting disjoint 64 MB blocks, and T threads memcpy-ing into a shared
// mapping of the file (ftruncate'd to size first).  Usage: wbench <path> <GB> <threads>
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

#define BLK (64ull << 20)
static uint8_t* src;
static uint64_t total;
static int T, fd;
static uint8_t* map;

static void* pw_worker(void* a) {
  int t = (int)(intptr_t)a;
  for (uint64_t b = (uint64_t)t * BLK; b < total; b += (uint64_t)T * BLK) {
    uint64_t n = total - b < BLK ? total - b : BLK;
    for (uint64_t d = 0; d < n;) {
      ssize_t w = pwrite(fd, src + d, n - d, (off_t)(b + d));
      if (w <= 0) { perror("pwrite"); exit(1); }
      d += (uint64_t)w;
    }
  }
  return NULL;
}

static void* mm_worker(void* a) {
  int t = (int)(intptr_t)a;
  for (uint64_t b = (uint64_t)t * BLK; b < total; b += (uint64_t)T * BLK) {
    uint64_t n = total - b < BLK ? total - b : BLK;
    memcpy(map + b, src, n);
  }
  return NULL;
}

static void run(const char* path, const char* name, void* (*fn)(void*), int threads, int use_map) {
  unlink(path);
  fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) { perror("open"); exit(1); }
  T = threads;
  double t0 = now();
  if (use_map) {
    if (ftruncate(fd, (off_t)total)) { perror("ftruncate"); exit(1); }
    map = mmap(NULL, total, PROT_WRITE, MAP_SHARED, fd, 0);
    if (map == MAP_FAILED) { perror("mmap"); exit(1); }
  }
  pthread_t th[64];
  for (int i = 0; i < T; i++) pthread_create(&th[i], NULL, fn, (void*)(intptr_t)i);
  for (int i = 0; i < T; i++) pthread_join(th[i], NULL);
  double t1 = now();
  if (use_map) munmap(map, total);
  close(fd);
  double t2 = now();
  printf("%-24s threads %2d: %.3f s (%.2f GB/s), close/unmap %.3f s\n", name, T, t1 - t0, total / (t1 - t0) / 1e9, t2 - t1);
  fflush(stdout);
  unlink(path);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  total = (uint64_t)(atof(argv[2]) * 1e9);
  int thr = atoi(argv[3]);
  src = aligned_alloc(4096, BLK);
  memset(src, 'a', BLK);
  for (uint64_t i = 0; i < BLK; i += 97) src[i] = '\n';
  run(argv[1], "pwrite 1 thread", pw_worker, 1, 0);
  run(argv[1], "pwrite threads", pw_worker, thr, 0);
  run(argv[1], "mmap memcpy threads", mm_worker, thr, 1);
  run(argv[1], "mmap memcpy 4 threads", mm_worker, 4, 1);
  run(argv[1], "pwrite 1 thread (again)", pw_worker, 1, 0);
  return 0;
}
