/*
 * CPU check of the request router's worker/device dispatch (kgx_dispatch.h),
 * run by tests/test_dispatch_native.py.  Prints "ok" or the first violation.
 *
 * Properties (kgx_server --devices spreads a request's pieces over GPUs):
 *  1. with W workers over D device slots and all idle, k <= D concurrent
 *     leases land on k distinct slots, in slot order 0, 1, 2, ...;
 *  2. the (D+1)-th lease goes back to slot 0, and in general no slot ever
 *     holds two more leases than another while the latter has idle workers;
 *  3. a slot-restricted lease (the mapping's device) only returns workers
 *     of that slot, and -1 when that slot has none idle;
 *  4. random lease/release sequences keep the busy counts consistent.
 */
#include <cstdio>
#include <random>
#include <vector>

#include "kgx_dispatch.h"

using kgx::WorkerPicker;

static int bad(const char *what, int a, int b)
{
    std::printf("FAIL %s (%d, %d)\n", what, a, b);
    return 1;
}

int main()
{
    for (int D = 1; D <= 8; D++)
        for (int W = D; W <= 3 * D + 2; W++) {
            WorkerPicker p(W, D);
            std::vector<long> got;
            for (int k = 0; k < W; k++) {
                long w = p.pick();
                if (w < 0)
                    return bad("no idle worker while some are idle", D, W);
                if (k < D && (int)p.slot_of(w) != k)
                    return bad("first leases not in slot order", D, k);
                /* balance: the chosen slot is among the least busy slots with an idle worker */
                for (int s = 0; s < D; s++) {
                    if (p.busy(s) < p.busy(p.slot_of(w)) && p.pick(s) >= 0)
                        return bad("lease skipped a less busy slot", D, s);
                }
                p.lease(w);
                got.push_back(w);
            }
            if (p.pick() != -1)
                return bad("a worker left idle after W leases", D, W);
            for (int s = 0; s < D; s++)
                if (p.pick(s) != -1)
                    return bad("restricted pick found a leased worker", D, s);
            /* release slot 0's workers: restricted and free picks return slot 0 */
            for (long w : got)
                if (p.slot_of(w) == 0)
                    p.release(w);
            long w0 = p.pick(0), wf = p.pick();
            if (w0 < 0 || p.slot_of(w0) != 0 || wf < 0 || p.slot_of(wf) != 0)
                return bad("restricted pick on a freed slot", D, W);
        }
    /* random sequences */
    std::mt19937 rng(7);
    for (int trial = 0; trial < 2000; trial++) {
        const int D = 1 + rng() % 8, W = D + rng() % 20;
        WorkerPicker p(W, D);
        std::vector<bool> leased(W, false);
        for (int step = 0; step < 200; step++) {
            if (rng() % 2) {
                const long only = rng() % 3 == 0 ? (long)(rng() % D) : -1;
                long w = p.pick(only);
                if (w >= 0) {
                    if (leased[w] || (only >= 0 && (long)p.slot_of(w) != only))
                        return bad("picked a leased or foreign worker", trial, step);
                    p.lease(w);
                    leased[w] = true;
                }
            } else {
                std::vector<int> ls;
                for (int w = 0; w < W; w++)
                    if (leased[w])
                        ls.push_back(w);
                if (!ls.empty()) {
                    int w = ls[rng() % ls.size()];
                    p.release(w);
                    leased[w] = false;
                }
            }
            for (int s = 0; s < D; s++) {
                size_t n = 0;
                for (int w = 0; w < W; w++)
                    n += leased[w] && (int)p.slot_of(w) == s;
                if (n != p.busy(s))
                    return bad("busy count drifted", trial, s);
            }
        }
    }
    std::printf("ok\n");
    return 0;
}
