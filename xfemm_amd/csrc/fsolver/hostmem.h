// Large host arrays of the product path on transparent huge pages.
//
// First-touching fresh anonymous memory costs ~20 ms per 128 MiB in 4 KiB
// page faults on the GPU box's host, ~1-7 ms when the range is advised for
// 2 MiB pages (THP there is in "madvise" mode; tools/lab/io_probe.cpp).  The
// FSolver path allocates a few hundred MiB per analysis (the mesh files, the
// element / node records, the renumbering keys, the .ans text), so every
// large array is advised before its first touch.
#pragma once

#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>

namespace xfemm {

constexpr size_t kHugePage = (size_t)2 << 20;

// advise the 2 MiB-aligned part of [p, p + bytes) for huge pages (no effect
// on a range already touched, nor where THP is off)
inline void advise_huge(void *p, size_t bytes)
{
    const uintptr_t a = ((uintptr_t)p + kHugePage - 1) & ~(uintptr_t)(kHugePage - 1);
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)(kHugePage - 1);
    if (e > a) (void)madvise((void *)a, e - a, MADV_HUGEPAGE);
}

// An allocator whose argument-less construct leaves the element untouched:
// resize() of a large array writes nothing, and the caller first-touches it
// in parallel (a sequential value-initialisation of ~100 MB costs ~5 ms of
// page faults and stores on one core).  For trivially destructible,
// trivially copyable records only.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U> &) noexcept
    {
    }
    template <class U>
    void construct(U *) noexcept
    {
    }
    template <class U, class A0, class... A>
    void construct(U *p, A0 &&a0, A &&...a)
    {
        ::new ((void *)p) U(std::forward<A0>(a0), std::forward<A>(a)...);
    }
};
template <class T>
using BigVec = std::vector<T, NoInitAlloc<T>>;

// reserve n elements of v, advised for huge pages when large, before the
// caller's assign / resize touches them
template <class T, class A>
void huge_reserve(std::vector<T, A> &v, size_t n)
{
    if (v.capacity() >= n) return;
    std::vector<T, A>().swap(v);
    v.reserve(n);
    if (n * sizeof(T) >= ((size_t)4 << 20)) advise_huge(v.data(), n * sizeof(T));
}

// an uninitialised buffer of trivially copyable T (2 MiB-aligned and advised
// when large)
template <class T>
struct HugeBuf {
    static_assert(std::is_trivially_copyable<T>::value, "raw buffer");
    T *p = nullptr;
    size_t n = 0;
    HugeBuf() = default;
    HugeBuf(const HugeBuf &) = delete;
    HugeBuf &operator=(const HugeBuf &) = delete;
    HugeBuf(HugeBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr, o.n = 0; }
    ~HugeBuf() { std::free(p); }
    // at least count elements (contents undefined); keeps a large enough buffer
    bool allocate(size_t count)
    {
        if (count <= n && p) return true;
        std::free(p);
        p = nullptr;
        n = 0;
        const size_t bytes = std::max<size_t>(1, count * sizeof(T));
        if (bytes >= ((size_t)4 << 20)) {
            p = static_cast<T *>(std::aligned_alloc(kHugePage, (bytes + kHugePage - 1) & ~(kHugePage - 1)));
            if (p) advise_huge(p, bytes);
        } else {
            p = static_cast<T *>(std::malloc(bytes));
        }
        if (p) n = count;
        return p != nullptr;
    }
    T *data() { return p; }
    const T *data() const { return p; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
};

}  // namespace xfemm
