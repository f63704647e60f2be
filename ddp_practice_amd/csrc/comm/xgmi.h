// One-shot xGMI all-reduce engine (implementation: comm/xgmi_allreduce.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <torch/extension.h>

#include <atomic>
#include <string>
#include <vector>

#include "comm/collective.h"
#include "comm/xsite.h"

namespace dpa {
namespace xgmi {

struct Peers {
  char* base[kMaxRanks];  // every rank's workspace, mapped into this process
};

// Host side of xsite_advance's limit: a launch whose workgroups on an active site
// outnumber the site's kEpochWords epoch words cannot advance every word by one, so the
// next launch on the site would re-use this epoch and read the peers' previous rows.
// Every launcher that attaches a site sets its workgroup count through this check.
inline bool site_grid_fits(long long nblk) { return nblk >= 1 && nblk <= kEpochWords; }
inline void set_site_grid(XSite& xs, long long nblk, const char* what) {
  if (!xs.active()) return;
  TORCH_CHECK(site_grid_fits(nblk), what, ": ", nblk, " workgroups on one in-kernel exchange site (at most ",
              kEpochWords, "); the caller must take the all-reduce launch path");
  xs.nblk = (int)nblk;
}

class XgmiComm {
 public:
  // max_bytes: largest message this engine takes; timeout_s: bound on every wait
  // max_bytes: largest one-shot message; twoshot_max_bytes: largest two-shot message (0: none)
  XgmiComm(int rank, int world, int device, long long max_bytes, double timeout_s, long long twoshot_max_bytes = 0);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;

  pybind11::bytes handle() const;               // IPC handle of this rank's workspace
  void open(std::vector<std::string> handles);  // map every peer's workspace
  void close();

  bool supports(const at::Tensor& t) const;
  // out may alias in; stream == nullptr: the caller's current stream
  void all_reduce(const at::Tensor& in, const at::Tensor& out, RedOp op, hipStream_t stream);
  // reduce-scatter + all-gather over direct peer writes (large messages)
  bool supports_twoshot(const at::Tensor& t) const;
  void all_reduce_twoshot(const at::Tensor& in, const at::Tensor& out, RedOp op, hipStream_t stream);
  long long twoshot_max_bytes() const { return ts_max_elems_ * 4; }  // as fp32
  void set_twoshot_blocks(int g);  // grid of every two-shot launch (before the first one)

  // test entry: `grid` workgroups exchange `in` through SyncBN site s (comm/xsite.h)
  void site_probe(int s, const at::Tensor& in, const at::Tensor& out, int grid);
  int error() const;  // 0 ok, 1 a peer never arrived (timeout), 2 aborted
  std::string error_string() const;
  void abort();       // every waiting block gives up (watchdog path)
  // Where this rank's exchanges stand: per used site the epoch its launches reached and the
  // epoch of the newest granule each peer pushed into this rank's rows (both parities), the
  // one-/two-shot block epochs and the error / abort words.  Read on a side thread through a
  // non-blocking stream, bounded by wait_s (a stuck compute stream cannot hold it up).
  std::string debug_state(double wait_s = 2.0) const;
  void set_timeout(double s) { timeout_ticks_ = (long long)(s * 1e8); }
  long long max_bytes() const { return max_elems_ * 4; }  // as fp32
  long long workspace_bytes() const { return ws_bytes_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  // in-kernel SyncBN exchange site s (comm/xsite.h) for this rank's kernels
  XSite site(int s) const;
  // the DDP gradient exchange of the fused AMP-SGD step (rows of max_bytes/4 floats)
  XSite grad_site() const;
  // the ResNet statistics finishers' site (rows of kWideVals floats; nblk set per launch)
  XSite wide_site() const;
  // test entry: `nblk` finisher workgroups each exchange a slice of `in` (<= kWideVals
  // floats) through the wide site with the positioned form; out = the global row
  void wide_probe(const at::Tensor& in, const at::Tensor& out, int nblk);
  long long max_elems() const { return max_elems_; }

 private:
  int rank_, world_, device_;
  long long max_elems_ = 0, slot_bytes_ = 0, ctr_off_ = 0, ws_bytes_ = 0, timeout_ticks_ = 0;
  int max_blocks_ = 0;
  char* local_ = nullptr;
  uint32_t* ctr_ = nullptr;  // per-block epoch counters: ordinary (cached) device memory
  unsigned long long* ticks_ = nullptr;  // per-site {epoch | tickets} words (ordinary device memory)
  long long site_off_ = 0;               // byte offset of the fused-site regions in every workspace
  long long grad_off_ = 0;               // byte offset of the gradient-exchange region
  long long wide_off_ = 0;               // byte offset of the wide site's region
  long long ts_off_ = 0, ts_par_bytes_ = 0, ts_shard_max_ = 0, ts_max_elems_ = 0;  // two-shot region
  int ts_blocks_ = 0, ts_grid_ = 0;
  bool ts_used_ = false;
  uint32_t* ts_ctr_ = nullptr;           // two-shot per-block epoch counters
  Peers peers_;
  int* host_words_ = nullptr;  // [0] error, [1] abort (host-mapped, coherent)
  int* dev_words_ = nullptr;
  bool opened_ = false;
  // what this rank's host has issued (debug_state, readable when the device is wedged):
  // launches attached to each site, one- / two-shot all-reduces and the last one's bytes
  mutable std::atomic<long long> site_calls_[kSites] = {};
  std::atomic<long long> ar_calls_{0}, ts_calls_{0}, ar_last_bytes_{0};
};

}  // namespace xgmi
}  // namespace dpa
