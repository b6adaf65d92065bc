// rtc_probe.cpp — development probe: compile one mixed-radix specialisation
// with hipRTC the way mixed_jit.hip does, print the log and timings.
//   hipcc -O2 rtc_probe.cpp -o rtc_probe -lhiprtc ; ./rtc_probe <arch> <incdir> <R...>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>
int main(int argc, char **argv) {
  std::string arch = argc > 1 ? argv[1] : "";
  if (arch == "dev") {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) != hipSuccess) return 2;
    arch = p.gcnArchName;
  }
  const std::string inc = std::string("-I") + (argc > 2 ? argv[2] : ".");
  std::string list;
  int n = 1;
  for (int i = 3; i < argc; ++i) { list += std::string(", ") + argv[i]; n *= atoi(argv[i]); }
  const std::string sp = n > 4096 ? "true" : "false", sw = atoi(argv[3]) % 2 == 0 ? "true" : "false";
  std::vector<std::string> names = {"&gdsp::fft_mixed_fixed_kernel<false, 0, " + sp + ", " + sw + list + ">",
                                    "&gdsp::pwelch_fixed_kernel<" + sw + list + ">"};
  hiprtcProgram prog;
  hiprtcCreateProgram(&prog, "#include \"mixed_fixed.hpp\"\n", "probe.hip", 0, nullptr, nullptr);
  for (auto &nm : names) hiprtcAddNameExpression(prog, nm.c_str());
  const std::string a = "--offload-arch=" + arch;
  const char *opts[] = {a.c_str(), "-O3", "-std=c++17", inc.c_str()};
  auto t0 = std::chrono::steady_clock::now();
  hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
  auto t1 = std::chrono::steady_clock::now();
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  std::string log(ls, 0);
  if (ls) hiprtcGetProgramLog(prog, &log[0]);
  printf("n=%d arch=%s rc=%d (%s) %.2f s\nlog[%zu]: %.3000s\n", n, arch.c_str(), (int)r,
         hiprtcGetErrorString(r), std::chrono::duration<double>(t1 - t0).count(), ls, log.c_str());
  return r == HIPRTC_SUCCESS ? 0 : 1;
}
