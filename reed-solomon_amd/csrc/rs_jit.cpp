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

namespace rsamd {

static const char* kArgsHeader =
#include "gen/rs_v1args_h.inc"
    ;
static const char* kDeviceHeader =
#include "gen/rs_device_h.inc"
    ;
// string literals of the generated call step (csrc/gen_asm.py v1_jitcall), as source text
static const char* kCallAsm =
#include "gen/v1_jitcall_text.inc"
    ;

struct JitModule {
    hipModule_t mod = nullptr;
    int device = 0;
    ~JitModule() {
        if (mod) (void)hipModuleUnload(mod);
    }
};

JitKernel::~JitKernel() {
    if (d_boff) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        (void)hipFree(d_boff);
        (void)hipSetDevice(cur);
    }
}

bool jit_supported(int m, int K, int R) {
    const int ntiles = (R + 31) / 32;
    return m <= 8 && K >= 1 && R >= 1 && int64_t(ntiles) * K <= kJitMaxBlocks;
}

std::string jit_source(const std::vector<uint8_t>& cg, int K, int R, std::vector<int32_t>* boff) {
    const int ntiles = (R + 31) / 32;
    std::ostringstream blk;
    int32_t off = 0;
    if (boff) boff->assign(size_t(ntiles) * K, 0);
    for (int t = 0; t < ntiles; ++t) {
        const int rows = std::min(32, R - 32 * t);
        for (int i = 0; i < K; ++i) {
            if (boff) (*boff)[size_t(t) * K + i] = off;
            for (int h = 0; h < 2; ++h)  // low nibbles (table v[8:23]), then high nibbles (v[24:39])
                for (int p = 0; p < rows; ++p) {
                    const int c = cg[size_t(32 * t + p) * K + i];
                    const int e = h ? c >> 4 : c & 15;
                    if (!e) continue;  // T[0] = 0
                    blk << "\"v_xor_b32 v" << 40 + p << ", v" << (h ? 24 : 8) + e << ", v" << 40 + p << "\\n\"\n";
                    off += 4;
                }
            blk << "\"s_setpc_b64 s[72:73]\\n\"\n";
            off += 4;
        }
    }
    std::ostringstream o;
    o << "#define RS_JIT_SOURCE 1\n"
         "typedef unsigned int uint32_t; typedef int int32_t; typedef unsigned short uint16_t;\n"
         "typedef unsigned char uint8_t; typedef long long int64_t; typedef unsigned long long uint64_t;\n"
         "typedef unsigned long uintptr_t;\n"
      << kArgsHeader << "\n"
      << kDeviceHeader << "\n"
      << "extern \"C\" __global__ void __launch_bounds__(256) rs_v1jit(V1Args a) {\n"
         "  __shared__ __attribute__((aligned(16))) uint32_t lds[V1_LDS_WORDS];\n"
         "  // lookup blocks of this matrix (entered only through s_swappc_b64 from the step below)\n"
         "  asm volatile(\"s_branch L_rs_blocks_end\\n\"\n"
         "\"L_rs_blk0:\\n\"\n"
      << blk.str()
      << "\"L_rs_blocks_end:\\n\"\n"
         "\".if (L_rs_blocks_end - L_rs_blk0) != "
      << off
      << "\\n\"\n"
         "\".error \\\"rs_v1jit: lookup block size mismatch\\\"\\n\"\n"
         "\".endif\\n\" ::: \"memory\");\n"
         "  m8_v1_run(a, lds, [&](uint32_t y, int i, int tile, u32x16& a0, u32x16& a1, const uint32_t*) {\n"
         "    const int off = sload(a.boff + tile * a.K + i);\n"
         "    const uint32_t k1d = 0x1D1D1D1Du;\n"
         "    uint32_t t0, t1;\n"
         "    u32x16 Tl, Th;\n"
         "    asm volatile(\n"
      << kCallAsm
      << "      : \"+{v[40:55]}\"(a0), \"+{v[56:71]}\"(a1), \"=&{v[8:23]}\"(Tl), \"=&{v[24:39]}\"(Th), [t0] \"=&v\"(t0),"
         " [t1] \"=&v\"(t1)\n"
         "      : [y0] \"v\"(y), [off] \"s\"(off), [k1d] \"v\"(k1d)\n"
         "      : \"s72\", \"s73\", \"s74\", \"s75\", \"scc\");\n"
         "  });\n"
         "}\n";
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
    if (hiprtcCreateProgram(&prog, src.c_str(), "rs_v1jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 1;
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
int jit_code(const std::string& src, const char* prefix, uint64_t h, std::vector<char>& code) {
    char name[48];
    std::snprintf(name, sizeof name, "%s_%016llx.co", prefix, static_cast<unsigned long long>(h));
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

uint64_t jit_hash(const std::string& s) { return fnv1a(s); }

static std::mutex g_jit_mu;
static std::map<std::pair<int, uint64_t>, std::shared_ptr<JitModule>> g_jit_mods;

int jit_module(const std::string& src, const char* prefix, std::shared_ptr<JitModule>& out, uint64_t* hash) {
    const uint64_t h = fnv1a(src);
    if (hash) *hash = h;
    int device = 0;
    (void)hipGetDevice(&device);
    std::lock_guard<std::mutex> lk(g_jit_mu);
    std::shared_ptr<JitModule>& slot = g_jit_mods[{device, h}];
    if (!slot) {
        std::vector<char> code;
        if (jit_code(src, prefix, h, code)) return 3;
        auto mod = std::make_shared<JitModule>();
        mod->device = device;
        hipError_t e = hipModuleLoadData(&mod->mod, code.data());
        if (e != hipSuccess) {
            std::fprintf(stderr, "librs_amd: hipModuleLoadData: %s\n", hipGetErrorString(e));
            return 3;
        }
        slot = mod;
    }
    out = slot;
    return 0;
}

hipModule_t jit_module_handle(const JitModule& m) { return m.mod; }

int jit_precompile(const std::vector<uint8_t>& cg, int K, int R) {
    if (!jit_supported(8, K, R)) return 0;
    const std::string src = jit_source(cg, K, R, nullptr);
    std::vector<char> code;
    return jit_code(src, "v1", fnv1a(src), code) ? 3 : 0;
}

int jit_build(const std::vector<uint8_t>& cg, int K, int R, std::unique_ptr<JitKernel>& out) {
    out.reset();
    if (!jit_supported(8, K, R)) return 0;
    std::vector<int32_t> boff;
    const std::string src = jit_source(cg, K, R, &boff);
    uint64_t h = 0;
    std::shared_ptr<JitModule> slot;
    if (jit_module(src, "v1", slot, &h)) return 3;
    int device = 0;
    (void)hipGetDevice(&device);
    auto k = std::make_unique<JitKernel>();
    k->mod = slot;
    k->device = device;
    k->ntiles = (R + 31) / 32;
    if (hipModuleGetFunction(&k->fn, slot->mod, "rs_v1jit") != hipSuccess) return 3;
    if (hipMalloc(&k->d_boff, boff.size() * 4) != hipSuccess) return 3;
    if (hipMemcpy(k->d_boff, boff.data(), boff.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 3;
    char nm[64];
    std::snprintf(nm, sizeof nm, "rs_v1jit[%dx%d:%08llx]", R, K, static_cast<unsigned long long>(h & 0xffffffff));
    k->name = nm;
    out = std::move(k);
    return 0;
}

int jit_launch(const JitKernel& k, V1Args v, int64_t n_stripes, hipStream_t st) {
    if (n_stripes <= 0 || v.nchunks <= 0) return 0;
    v.boff = k.d_boff;
    void* args[] = {&v};
    hipError_t e = hipModuleLaunchKernel(k.fn, unsigned(n_stripes * v.nchunks), unsigned(k.ntiles), 1, 256, 1, 1, 0,
                                         st, args, nullptr);
    if (e != hipSuccess) {
        std::fprintf(stderr, "librs_amd: jit launch: %s\n", hipGetErrorString(e));
        return 3;
    }
    return 0;
}

}  // namespace rsamd
