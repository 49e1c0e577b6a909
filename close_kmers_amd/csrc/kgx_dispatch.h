/*
 * kgx_dispatch.h -- which KmerGuts worker (hence which GPU) a request piece
 * runs on.  Header-only, no HIP: the request router uses it, and
 * tests/native/dispatch_check.cpp checks the order on the CPU.
 *
 * The reference's pool hands tasks to whichever of its threads is free, all
 * over one image (threadpool.cc:18-44).  Here worker w holds a context on the
 * image replica of device slot w % n_slots, so "whichever is free" decides
 * which GPU does the work.  The rule spreads concurrent work over the
 * devices: lease the idle worker whose slot has the fewest leased workers
 * (ties: the lowest slot), and on that slot the lowest-numbered idle worker.
 * So n concurrent pieces of a large request land on n different GPUs while
 * there are idle GPUs, and a device gets a second worker only when every
 * device is busy.  A lease may be restricted to one slot (handlers whose
 * device tables live on the mapping's device).
 */
#pragma once

#include <cstddef>
#include <vector>

namespace kgx {

class WorkerPicker {
public:
    WorkerPicker(size_t n_workers, size_t n_slots)
        : slot_(n_workers), idle_(n_workers, true), busy_(n_slots ? n_slots : 1, 0)
    {
        for (size_t w = 0; w < n_workers; w++)
            slot_[w] = w % busy_.size();
    }
    size_t n_workers() const { return slot_.size(); }
    size_t n_slots() const { return busy_.size(); }
    size_t slot_of(size_t w) const { return slot_[w]; }
    size_t busy(size_t slot) const { return busy_[slot]; }

    /* the worker to lease next (-1 when none is idle); only_slot >= 0
     * restricts the choice to that slot's workers */
    long pick(long only_slot = -1) const
    {
        long best = -1;
        for (size_t w = 0; w < slot_.size(); w++) {
            if (!idle_[w] || (only_slot >= 0 && slot_[w] != (size_t)only_slot))
                continue;
            if (best < 0 || busy_[slot_[w]] < busy_[slot_[(size_t)best]] ||
                (busy_[slot_[w]] == busy_[slot_[(size_t)best]] && slot_[w] < slot_[(size_t)best]))
                best = (long)w;
        }
        return best;
    }
    void lease(size_t w)
    {
        idle_[w] = false;
        busy_[slot_[w]]++;
    }
    void release(size_t w)
    {
        idle_[w] = true;
        busy_[slot_[w]]--;
    }

private:
    std::vector<size_t> slot_;
    std::vector<bool> idle_;
    std::vector<size_t> busy_;
};

}  // namespace kgx
