// test_per_device.cpp -- the keying of per-GPU library state
// (draid-spdk_amd/csrc/per_device.hpp), on the CPU: a slot per device ordinal,
// independent of the others, nothing for an ordinal out of range; and which GPU a
// resolved address range may be used on.
#include <cstdio>
#include <cstdlib>

#include "../../draid-spdk_amd/csrc/per_device.hpp"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                     \
        }                                                                \
    } while (0)

struct Scratch {  // shaped like the library's: a buffer owned by one GPU
    void* arena = nullptr;
    int allocated_on = -1;
};

// What a call does: take the current GPU's slot, allocate there on first use.
static Scratch* use(draid::PerDevice<Scratch>& all, int current_device)
{
    Scratch* s = all.at(current_device);
    if (s && !s->arena) {
        s->arena = malloc(16);
        s->allocated_on = current_device;
    }
    return s;
}

int main()
{
    draid::PerDevice<Scratch> all;
    // a thread that works on GPU 0, then 1, then 0 again
    Scratch* a = use(all, 0);
    Scratch* b = use(all, 1);
    Scratch* c = use(all, 0);
    CHECK(a && b && a != b && a == c);
    CHECK(a->allocated_on == 0 && b->allocated_on == 1);  // never GPU 0's arena on GPU 1
    CHECK(a->arena != b->arena);
    for (int d = 0; d < draid::kMaxDevices; ++d) {
        Scratch* s = use(all, d);
        CHECK(s && s->allocated_on == d && s == all.at(d));
    }
    CHECK(all.at(-1) == nullptr && all.at(draid::kMaxDevices) == nullptr);
    const draid::PerDevice<Scratch>& view = all;
    CHECK(view.at(3) == all.at(3));
    for (int d = 0; d < draid::kMaxDevices; ++d)
        free(all.at(d)->arena);

    // address ranges: host memory anywhere, device memory on its own GPU only
    using draid::kAnyDevice;
    using draid::range_usable_on;
    static_assert(range_usable_on(kAnyDevice, 0) && range_usable_on(kAnyDevice, 7), "host memory");
    static_assert(range_usable_on(2, 2), "own GPU");
    static_assert(!range_usable_on(0, 1) && !range_usable_on(1, 0), "another GPU's memory");
    static_assert(range_usable_on(5, kAnyDevice), "caller did not say where the kernel runs");
    CHECK(!range_usable_on(0, 1));
    printf("PASS per-device keying\n");
    return 0;
}
