// TEST INFRASTRUCTURE ONLY. Driver for the REFERENCE diff() (gallocy/utils/diff.cpp:73-167),
// compiled by oracle/Makefile straight from the sources under /root/reference into
// oracle/_ref/ref_nw_driver. No reference source is copied into this repository.
//
// Modes:
//   ref_nw_driver run  <cases.bin> <out.bin>
//       cases.bin: repeated [u32 n1][u32 n2][n1 bytes][n2 bytes]; inputs must not contain NUL
//       (the reference returns NUL-terminated alignments and no length, diff.h:9-11).
//       out.bin:   repeated [u32 L][L bytes out1][L bytes out2]; L = strlen(out1) (== strlen(out2)
//       is checked). Each case runs in a forked child so the reference's single 32 MiB internal
//       zone (utils/constants.h:11) starts fresh, as in a new test binary.
//   ref_nw_driver time <n> <reps>
//       Times the reference diff() on two n-byte random strings (10 % substitutions,
//       test/test_diff.cpp:38-57 style), one forked child per rep, prints "seconds_per_call cells".
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gallocy/allocators/internal.h"
#include "gallocy/utils/diff.h"

// constants.cpp:7 declares `extern char* main;`, which g++ >= 11 rejects; the Makefile compiles
// it with -Dmain=__gallocy_main_anchor. The variable is only read by global_main(), which is
// not on the diff path; this is its definition.
extern "C" {
char* __gallocy_main_anchor;
}

static int run_case(const std::vector<char>& a, const std::vector<char>& b, int out_fd) {
  char* o1 = nullptr;
  char* o2 = nullptr;
  int ret = diff(a.data(), a.size(), o1, b.data(), b.size(), o2);
  if (ret != 0) return 2;
  uint32_t L1 = (uint32_t)strlen(o1), L2 = (uint32_t)strlen(o2);
  if (L1 != L2) return 3;
  if (write(out_fd, &L1, 4) != 4) return 4;
  if (L1 && write(out_fd, o1, L1) != (ssize_t)L1) return 4;
  if (L1 && write(out_fd, o2, L1) != (ssize_t)L1) return 4;
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 4 && !strcmp(argv[1], "run")) {
    FILE* in = fopen(argv[2], "rb");
    FILE* out = fopen(argv[3], "wb");
    if (!in || !out) return 1;
    fflush(out);
    for (;;) {
      uint32_t n1, n2;
      if (fread(&n1, 4, 1, in) != 1) break;
      if (fread(&n2, 4, 1, in) != 1) return 1;
      std::vector<char> a(n1 + 1, 0), b(n2 + 1, 0);
      if (n1 && fread(a.data(), 1, n1, in) != n1) return 1;
      if (n2 && fread(b.data(), 1, n2, in) != n2) return 1;
      a.resize(n1);
      b.resize(n2);
      fflush(out);
      pid_t pid = fork();
      if (pid == 0) _exit(run_case(a, b, fileno(out)));
      int st = 0;
      waitpid(pid, &st, 0);
      if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
        fprintf(stderr, "case n1=%u n2=%u failed (status %d)\n", n1, n2, st);
        return 5;
      }
    }
    fclose(out);
    return 0;
  }
  if (argc >= 4 && !strcmp(argv[1], "time")) {
    const int n = atoi(argv[2]);
    const int reps = atoi(argv[3]);
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
      int fds[2];
      if (pipe(fds)) return 1;
      pid_t pid = fork();
      if (pid == 0) {
        srand(1234 + r);
        std::vector<char> a(n), b(n);
        for (int i = 0; i < n; ++i) a[i] = (char)(1 + rand() % 254);
        b = a;
        for (int i = 0; i < n; ++i)
          if (rand() % 10 == 1) b[i] = (char)(1 + rand() % 254);
        char* o1 = nullptr;
        char* o2 = nullptr;
        auto t0 = std::chrono::steady_clock::now();
        diff(a.data(), n, o1, b.data(), n, o2);
        auto t1 = std::chrono::steady_clock::now();
        double s = std::chrono::duration<double>(t1 - t0).count();
        if (write(fds[1], &s, sizeof(s)) != sizeof(s)) _exit(1);
        _exit(0);
      }
      close(fds[1]);
      double s = 0;
      ssize_t got = read(fds[0], &s, sizeof(s));
      close(fds[0]);
      int st = 0;
      waitpid(pid, &st, 0);
      if (got != sizeof(s) || !WIFEXITED(st) || WEXITSTATUS(st) != 0) return 6;
      if (s < best) best = s;
    }
    printf("%.9f %llu\n", best, (unsigned long long)n * (unsigned long long)n);
    return 0;
  }
  fprintf(stderr, "usage: %s run <cases> <out> | time <n> <reps>\n", argv[0]);
  return 1;
}
