// Minimal reproducer for the fault at process exit under rocprofv3 (VERDICT r04 "exit SIGSEGV"): no
// libkgpu, no torch -- one trivial kernel launched either as an ordinary dispatch or through
// hipLaunchCooperativeKernel, a synchronize, and a normal exit.  A SIGSEGV handler prints every frame
// with dladdr (library, symbol, offset from the library base) and the /proc/self/maps line holding it.
//   coop_exit_probe plain|coop [reset]
//     reset: hipDeviceReset() before returning from main
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void k_fill(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

static void maps_line(void* addr) {
  char buf[1 << 16];
  const int fd = open("/proc/self/maps", O_RDONLY);
  if (fd < 0) return;
  const ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return;
  buf[n] = 0;
  for (char* line = strtok(buf, "\n"); line; line = strtok(nullptr, "\n")) {
    unsigned long lo = 0, hi = 0;
    if (sscanf(line, "%lx-%lx", &lo, &hi) == 2 && (unsigned long)addr >= lo && (unsigned long)addr < hi) {
      fprintf(stderr, "      maps: %s\n", line);
      return;
    }
  }
}

static void on_segv(int sig, siginfo_t* si, void*) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  fprintf(stderr, "coop_exit_probe: signal %d at address %p, %d frames\n", sig, si ? si->si_addr : nullptr, n);
  for (int i = 0; i < n; ++i) {
    Dl_info d{};
    if (dladdr(fr[i], &d) && d.dli_fname) {
      fprintf(stderr, "  #%d %p %s(%s+0x%lx) base %p +0x%lx\n", i, fr[i], d.dli_fname, d.dli_sname ? d.dli_sname : "?",
              d.dli_saddr ? (unsigned long)((char*)fr[i] - (char*)d.dli_saddr) : 0ul, d.dli_fbase,
              (unsigned long)((char*)fr[i] - (char*)d.dli_fbase));
    } else {
      fprintf(stderr, "  #%d %p ?\n", i, fr[i]);
    }
    maps_line(fr[i]);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int main(int argc, char** argv) {
  struct sigaction sa {};
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, nullptr);
  const bool coop = argc > 1 && std::strcmp(argv[1], "coop") == 0;
  const bool reset = argc > 2 && std::strcmp(argv[2], "reset") == 0;
  int* d = nullptr;
  int n = 1 << 12;
  if (hipMalloc(&d, n * sizeof(int)) != hipSuccess) return 1;
  if (coop) {
    void* args[] = {(void*)&d, (void*)&n};
    if (hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_fill), dim3(n / 256), dim3(256), args, 0, 0) !=
        hipSuccess)
      return 2;
  } else {
    hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, d, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  int h = 0;
  if (hipMemcpy(&h, d + 77, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  std::printf("coop_exit_probe %s%s: %d\n", coop ? "coop" : "plain", reset ? " reset" : "", h);
  std::fflush(stdout);
  if (reset) (void)hipDeviceReset();
  return h == 77 ? 0 : 5;
}
