// Registration-churn probe for the round-3 fault ("registered caller symbols").
//
// Replays the allocator sequence of the round-3 symbol_create / symbol_destroy code before commit 5e60e5f
// (aligned_alloc in whole pages, hipHostRegister mapped + portable at creation, zero-copy kernel writes
// through the device-visible address, hipHostUnregister, free) and records what the runtime reports at
// each step, without ever copying into memory that reuses a freed range (that copy is the faulting
// action; this probe only asks the runtime about its state):
//   * the return code of every hipHostRegister / hipHostGetDevicePointer / hipHostUnregister;
//   * whether the device-visible address equals the host address (the GPU maps the pages at the CPU VA);
//   * hipPointerGetAttributes at the first, a middle and the last byte right after the unregister;
//   * for pageable buffers malloc'd after the frees (sizes of torch / numpy host tensors), which of their
//     pages overlap a once-registered range and what the runtime reports for each such page.
// Prints one JSON line. usage: reg_probe [rounds] [seed]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

__global__ void k_touch(uint32_t* p, size_t n, uint32_t v) {
    const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v ^ uint32_t(i);
}


static int attr_type(const void* p) {
    hipPointerAttribute_t at{};
    const hipError_t e = hipPointerGetAttributes(&at, p);
    (void)hipGetLastError();
    if (e != hipSuccess) return -1 - int(e);  // unknown to the runtime (an error code)
    return int(at.type);                      // hipMemoryTypeUnregistered = 0
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 40;
    std::srand(argc > 2 ? std::atoi(argv[2]) : 7);
    const size_t kPage = 4096;
    long reg_calls = 0, reg_fail = 0, getdev_fail = 0, dev_ne_host = 0, unreg_fail = 0, touch_bad = 0;
    long stale_after_unreg = 0, reuse_pages = 0, reuse_known = 0, reuse_bufs = 0, bufs = 0;
    long first_stale_type = 0;
    std::map<uintptr_t, uintptr_t> once;  // every range ever registered: start -> end (ranges may be re-registered)
    for (int round = 0; round < rounds; ++round) {
        // a big pageable allocation freed first raises glibc's dynamic mmap threshold, as the fuzz's numpy
        // arrays do, so later multi-MiB buffers come from the heap the symbols went back to
        void* big = std::malloc(size_t(8) << 20);
        std::memset(big, 1, size_t(8) << 20);
        std::free(big);
        const int nsym = 20 + std::rand() % 300;
        const size_t S = 16 * size_t(1024 + std::rand() % 3073);  // 16 .. 64 KiB, as fuzz dropin_reg
        const size_t bytes = (S + kPage - 1) / kPage * kPage;
        std::vector<uint8_t*> p(nsym);
        std::vector<uint32_t*> d(nsym, nullptr);
        std::vector<char> reg(nsym, 0);
        for (int i = 0; i < nsym; ++i) {
            p[i] = static_cast<uint8_t*>(std::aligned_alloc(kPage, bytes));
            std::memset(p[i], 0, bytes);
            ++reg_calls;
            if (hipHostRegister(p[i], bytes, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess) {
                ++reg_fail;
                (void)hipGetLastError();
                continue;
            }
            reg[i] = 1;
            once[uintptr_t(p[i])] = std::max(once[uintptr_t(p[i])], uintptr_t(p[i]) + bytes);
            void* dv = nullptr;
            if (hipHostGetDevicePointer(&dv, p[i], 0) != hipSuccess) {
                ++getdev_fail;
                (void)hipGetLastError();
                continue;
            }
            if (dv != p[i]) ++dev_ne_host;
            d[i] = static_cast<uint32_t*>(dv);
        }
        for (int i = 0; i < nsym; ++i)
            if (d[i]) k_touch<<<dim3(unsigned((S / 4 + 255) / 256)), dim3(256)>>>(d[i], S / 4, uint32_t(round * 977 + i));
        if (hipDeviceSynchronize() != hipSuccess) {
            std::printf("{\"error\": \"zero-copy kernel failed\"}\n");
            return 1;
        }
        for (int i = 0; i < nsym; ++i)
            if (d[i]) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(p[i]);
                if (w[0] != uint32_t(round * 977 + i) || w[S / 4 - 1] != (uint32_t(round * 977 + i) ^ uint32_t(S / 4 - 1)))
                    ++touch_bad;
            }
        for (int i = 0; i < nsym; ++i) {
            if (reg[i]) {
                const hipError_t e = hipHostUnregister(p[i]);
                (void)hipGetLastError();
                if (e != hipSuccess) ++unreg_fail;
            }
            const int t0 = attr_type(p[i]), t1 = attr_type(p[i] + bytes / 2), t2 = attr_type(p[i] + bytes - 1);
            if (t0 > 0 || t1 > 0 || t2 > 0) {
                if (!stale_after_unreg) first_stale_type = t0 > 0 ? t0 : (t1 > 0 ? t1 : t2);
                ++stale_after_unreg;
            }
            std::free(p[i]);
        }
        // pageable buffers of host-tensor sizes: which pages lie in a once-registered range, and what the
        // runtime says about them
        const int nb = 4 + std::rand() % 8;
        std::vector<uint8_t*> b(nb);
        for (int j = 0; j < nb; ++j) {
            const size_t sz = size_t(256) << 10 << (std::rand() % 5);  // 256 KiB .. 4 MiB
            b[j] = static_cast<uint8_t*>(std::malloc(sz));
            ++bufs;
            bool hit = false;
            for (size_t off = 0; off < sz; off += kPage) {
                const uintptr_t a = uintptr_t(b[j]) + off;
                auto it = once.upper_bound(a);
                bool in = false;
                for (int back = 0; back < 16 && it != once.begin(); ++back) {  // ranges are <= 64 KiB
                    --it;
                    if (a < it->second) { in = true; break; }
                }
                if (!in) continue;
                hit = true;
                ++reuse_pages;
                if (attr_type(b[j] + off) > 0) ++reuse_known;
            }
            reuse_bufs += hit;
        }
        for (int j = 0; j < nb; ++j) std::free(b[j]);
    }
    std::printf("{\"probe\": \"reg_churn\", \"rounds\": %d, \"register_calls\": %ld, \"register_failures\": %ld, "
                "\"get_device_pointer_failures\": %ld, \"device_ptr_ne_host\": %ld, \"zero_copy_bad\": %ld, "
                "\"unregister_failures\": %ld, \"attr_known_after_unregister\": %ld, \"first_stale_type\": %ld, "
                "\"pageable_bufs\": %ld, \"bufs_reusing_registered_pages\": %ld, \"reused_pages\": %ld, "
                "\"reused_pages_known_to_runtime\": %ld}\n",
                rounds, reg_calls, reg_fail, getdev_fail, dev_ne_host, touch_bad, unreg_fail, stale_after_unreg,
                first_stale_type, bufs, reuse_bufs, reuse_pages, reuse_known);
    return 0;
}
