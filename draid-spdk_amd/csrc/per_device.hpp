// per_device.hpp -- state that lives in one GPU's memory, kept per GPU.
//
// A process may drive several GPUs from one thread (draid_ec_set_device, the
// contexts of a raid module's channel, draid_ec_mgpu).  Scratch a call keeps
// between invocations -- a staging arena, a pointer table, a flag word -- is
// device memory of the GPU it was allocated on, and a kernel on another GPU that
// is handed its address takes a memory fault (no peer access is set up here).
// The relinked reference would hit exactly that: raid5_xor_buf
// (module/bdev/raid/raid5.c:188-201) calls xor_gen from whichever reactor, with
// whichever device that thread last selected.  So such state is indexed by the
// device ordinal, and a resolved address range remembers which GPU it is good
// for.  Pure host logic: no HIP call in here.
#pragma once

namespace draid {

constexpr int kMaxDevices = 16;

// One T per GPU, indexed by device ordinal.
template <class T>
struct PerDevice {
    T slot[kMaxDevices];

    // The slot of `device`, or nullptr for an ordinal outside [0, kMaxDevices).
    T* at(int device) { return device >= 0 && device < kMaxDevices ? &slot[device] : nullptr; }
    const T* at(int device) const
    {
        return device >= 0 && device < kMaxDevices ? &slot[device] : nullptr;
    }
};

// Where a resolved address range lives: kAnyDevice for pinned / registered host
// memory (mapped portably: every GPU reaches it), else the owning GPU's ordinal.
constexpr int kAnyDevice = -1;

// May a kernel running on GPU `on_device` use a range that lives on
// `range_device`?  on_device == kAnyDevice: the caller does not say (no check).
constexpr bool range_usable_on(int range_device, int on_device)
{
    return range_device == kAnyDevice || on_device == kAnyDevice || range_device == on_device;
}

}  // namespace draid
