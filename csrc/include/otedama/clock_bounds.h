// Device clock -> host clock from one-sided bounds. Every launch's probe stamp (s_memrealtime) is seen by the host
// some time after the device wrote it, so (host time after the load that saw it) - (stamp / f) bounds the offset
// between the clocks from above. The lowest bound of the last `window` seconds is the estimate: with ~5 launches a
// second it sits within a poll interval of the true offset, and the window lets it follow drift between the clocks.
// A monotonic deque keeps the window minimum in O(1) amortized per sample.
#pragma once
#include <deque>
#include <utility>

namespace otedama {

class ClockBounds {
 public:
  explicit ClockBounds(double window_s) : window_(window_s) {}

  // One sighting at host time `now` with offset bound `bound`; returns the window minimum after adding it.
  double add(double now, double bound) {
    while (!q_.empty() && q_.back().second >= bound) q_.pop_back();  // bounds increase from front to back
    q_.emplace_back(now, bound);
    while (now - q_.front().first > window_) q_.pop_front();  // the newest always stays
    return q_.front().second;
  }

  bool empty() const { return q_.empty(); }
  double min() const { return q_.front().second; }

 private:
  double window_;
  std::deque<std::pair<double, double>> q_;  // (seen at, bound), oldest first
};

}  // namespace otedama
