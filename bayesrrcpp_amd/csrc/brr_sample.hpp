// brr_sample.hpp -- the one-shot samplers' output pipeline (replaces the reference's
// moodycamel::ConcurrentQueue of VectorXd samples, src/BayesRv2.cpp:62,257-290).
//
// A ring of `depth` sample slots per session.  push() snapshots the chain's state into the next
// free slot's device buffer (device-to-device copies on the session stream, so the next sweep can
// start at once) and queues the slot's copy into pinned host memory on a copy stream; the writer
// thread waits for that copy, formats the row straight from pinned memory and releases the slot.
// When every slot is taken push() blocks, so a writer slower than the sampler throttles it
// instead of growing memory (the reference's queue is unbounded).
#pragma once
#include <stdint.h>

#include "../../include/brr.h"
#include "brr_device.hpp"

struct brr_session;

namespace brr {

struct SampleView {
  const Scal *sc;      // mu, sigmaE, tau, sigmaF, ...
  const double *beta;  // [M]
  const double *eps;   // [N]
  const double *lam;   // [M] (Horseshoe)
  const double *sgg;   // [G] sigmaGG
  const double *alpha; // [F]
  const int32_t *comp; // [M]
};

int sample_ring_open(brr_session *s, int depth);
int sample_ring_push(brr_session *s, int *slot);  // snapshot of the current state
int sample_ring_wait(brr_session *s, int slot, SampleView *v);  // its host copy is complete
void sample_ring_release(brr_session *s, int slot);
void sample_ring_close(brr_session *s);
int sample_ring_max_in_use(brr_session *s);  // diagnostics: most slots ever taken at once

// n sweeps as brr_session_sweep (single-GPU sessions), with the device error check (a stream sync and
// a read-back of the hand-over words) only when `check` is set: the one-shots check every few
// iterations instead of after each sweep, so the host keeps the device queue full
int session_sweep(brr_session *s, int n, bool check);

// a caller's options over the defaults, by the caller's ABI version: an older caller's struct
// ends before the fields a later ABI added (ABI 1: row shards, ABI 2: exchanges_per_sweep)
brr_options options_from_caller(const brr_options *in);

}  // namespace brr
