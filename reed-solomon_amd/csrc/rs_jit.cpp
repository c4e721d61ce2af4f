// rs_jit.cpp -- see rs_jit.hpp.
#include "rs_jit.hpp"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>

#include "gf16.hpp"

namespace rsamd {

static const char* kDeviceHeader =
#include "gen/rs_device_h.inc"
    ;

struct JitModule {
    hipModule_t mod = nullptr;
    int device = 0;
    ~JitModule() {
        if (mod) (void)hipModuleUnload(mod);
    }
};

bool jit_supported(int m, int K, int R) {
    return m <= 8 && R >= 1 && R <= kJitMaxRows && int64_t(K) * R <= kJitMaxPairs;
}

std::string jit_source(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                       const std::vector<int32_t>& out_slots) {
    const Gamma8& g = gamma8();
    std::ostringstream o;
    o << "#define RS_JIT_SOURCE 1\n"
         "typedef unsigned int uint32_t; typedef unsigned short uint16_t; typedef unsigned char uint8_t;\n"
         "typedef long long int64_t;\n"
      << kDeviceHeader << "\n";
    o << "extern \"C\" __global__ void __launch_bounds__(256) rs_jit_apply(const uint8_t* __restrict__ src,"
         " int64_t src_stripe, int64_t src_sym, uint8_t* __restrict__ dst, int64_t dst_stripe, int64_t dst_sym,"
         " const uint32_t* __restrict__ ltab, int64_t nbytes, int64_t nchunks) {\n"
         "  __shared__ uint32_t lt[2048];\n"
         "  for (int i = threadIdx.x; i < 2048; i += 256) lt[i] = ltab[i];\n"
         "  __syncthreads();\n"
         "  const int64_t stripe = int64_t(blockIdx.x) / nchunks;\n"
         "  const int64_t col = (int64_t(blockIdx.x) - stripe * nchunks) * 2048 + int64_t(threadIdx.x) * 8;\n"
         "  const int64_t avail = nbytes - col;\n"
         "  if (avail <= 0) return;\n"
         "  const uint8_t* s = src + stripe * src_stripe + col;\n";
    for (int p = 0; p < R; ++p) o << "  uint32_t a" << p << "_0 = 0, a" << p << "_1 = 0;\n";
    if (K > 0) o << "  uint32_t x[2], nx[2];\n  load_slice<8>(x, s + " << in_slots[0] << "LL * src_sym, avail);\n";
    for (int i = 0; i < K; ++i) {
        o << "  {\n";
        if (i + 1 < K) o << "    load_slice<8>(nx, s + " << in_slots[i + 1] << "LL * src_sym, avail);\n";
        for (int v = 0; v < 2; ++v) {
            o << "    const uint32_t m" << v << "0 = lds_lookup4(lt, x[" << v << "]);\n";
            for (int j = 1; j < 8; ++j) o << "    const uint32_t m" << v << j << " = xt8(m" << v << (j - 1) << ");\n";
        }
        for (int p = 0; p < R; ++p) {
            const uint32_t c = g.coord(M[size_t(p) * K + i]);
            int bits[8], nb = 0;
            for (int j = 0; j < 8; ++j)
                if (c & (1u << j)) bits[nb++] = j;
            for (int v = 0; v < 2; ++v) {
                int q = 0;
                for (; q + 1 < nb; q += 2)
                    o << "    a" << p << "_" << v << " = xor3(a" << p << "_" << v << ", m" << v << bits[q] << ", m" << v
                      << bits[q + 1] << ");\n";
                if (q < nb) o << "    a" << p << "_" << v << " ^= m" << v << bits[q] << ";\n";
            }
        }
        if (i + 1 < K) o << "    x[0] = nx[0]; x[1] = nx[1];\n";
        o << "  }\n";
    }
    o << "  uint8_t* d = dst + stripe * dst_stripe + col;\n";
    for (int p = 0; p < R; ++p)
        o << "  { uint32_t y[2] = {lds_lookup4(lt + 1024, a" << p << "_0), lds_lookup4(lt + 1024, a" << p
          << "_1)}; store_slice<8>(d + " << out_slots[p] << "LL * dst_sym, y, avail); }\n";
    o << "}\n";
    return o.str();
}

static uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
    return h;
}

static std::string cache_dir() {
    if (const char* e = std::getenv("RS_AMD_JIT_CACHE")) return e;
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(&jit_supported), &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t slash = p.rfind('/');
        if (slash != std::string::npos) return p.substr(0, slash) + "/jit_cache";
    }
    return "";
}

static int compile(const std::string& src, std::vector<char>& code) {
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "rs_jit_apply.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 1;
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
    if (r != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        std::fprintf(stderr, "librs_amd: hiprtc compile failed: %s\n%s\n", hiprtcGetErrorString(r), log.c_str());
        hiprtcDestroyProgram(&prog);
        return 1;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    code.resize(n);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    return 0;
}

// Code object for `src` from the disk cache, else compiled with hiprtc and stored there.
static int jit_code(const std::string& src, uint64_t h, std::vector<char>& code) {
    char name[32];
    std::snprintf(name, sizeof name, "%016llx.co", static_cast<unsigned long long>(h));
    const std::string dir = cache_dir();
    if (!dir.empty()) {
        std::ifstream f(dir + "/" + name, std::ios::binary);
        if (f) code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    }
    if (!code.empty()) return 0;
    if (compile(src, code)) return 1;
    if (!dir.empty()) {
        mkdir(dir.c_str(), 0755);
        const std::string tmp = dir + "/" + name + ".tmp" + std::to_string(getpid());
        std::ofstream f(tmp, std::ios::binary);
        if (f.write(code.data(), std::streamsize(code.size()))) {
            f.close();
            std::rename(tmp.c_str(), (dir + "/" + name).c_str());
        }
    }
    return 0;
}

int jit_precompile(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
                   const std::vector<int32_t>& out_slots) {
    if (!jit_supported(8, K, R)) return 0;
    const std::string src = jit_source(M, K, R, in_slots, out_slots);
    std::vector<char> code;
    return jit_code(src, fnv1a(src), code) ? 3 : 0;
}

static std::mutex g_jit_mu;
static std::map<std::pair<int, uint64_t>, std::shared_ptr<JitModule>> g_jit_mods;

int jit_build(const std::vector<uint16_t>& M, int K, int R, const std::vector<int32_t>& in_slots,
              const std::vector<int32_t>& out_slots, std::unique_ptr<JitKernel>& out) {
    out.reset();
    if (!jit_supported(8, K, R)) return 0;
    const std::string src = jit_source(M, K, R, in_slots, out_slots);
    const uint64_t h = fnv1a(src);
    int device = 0;
    (void)hipGetDevice(&device);
    std::lock_guard<std::mutex> lk(g_jit_mu);
    std::shared_ptr<JitModule>& slot = g_jit_mods[{device, h}];
    if (!slot) {
        std::vector<char> code;
        if (jit_code(src, h, code)) return 3;
        auto mod = std::make_shared<JitModule>();
        mod->device = device;
        hipError_t e = hipModuleLoadData(&mod->mod, code.data());
        if (e != hipSuccess) {
            std::fprintf(stderr, "librs_amd: hipModuleLoadData: %s\n", hipGetErrorString(e));
            return 3;
        }
        slot = mod;
    }
    auto k = std::make_unique<JitKernel>();
    k->mod = slot;
    if (hipModuleGetFunction(&k->fn, slot->mod, "rs_jit_apply") != hipSuccess) return 3;
    char nm[64];
    std::snprintf(nm, sizeof nm, "rs_jit_apply[%dx%d:%08llx]", R, K, static_cast<unsigned long long>(h & 0xffffffff));
    k->name = nm;
    out = std::move(k);
    return 0;
}

int jit_launch(const JitKernel& k, const uint8_t* src, int64_t src_stripe, int64_t src_sym, uint8_t* dst,
               int64_t dst_stripe, int64_t dst_sym, int64_t n_stripes, int64_t nbytes, const uint32_t* ltab,
               hipStream_t st) {
    int64_t nchunks = (nbytes + 2047) / 2048;
    if (n_stripes <= 0 || nchunks <= 0) return 0;
    void* args[] = {&src, &src_stripe, &src_sym, &dst, &dst_stripe, &dst_sym, &ltab, &nbytes, &nchunks};
    hipError_t e = hipModuleLaunchKernel(k.fn, unsigned(n_stripes * nchunks), 1, 1, 256, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) {
        std::fprintf(stderr, "librs_amd: jit launch: %s\n", hipGetErrorString(e));
        return 3;
    }
    return 0;
}

}  // namespace rsamd
