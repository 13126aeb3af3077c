"""Dashboard rendering (internal/tui/{dashboard,formatters}_test.go)."""
import io
import time

import pytest

from otedama_amd import tui


@pytest.mark.parametrize("hps,want", [(0, "0 H/s"), (999, "999 H/s"), (1500, "1.50 kH/s"), (2.5e6, "2.50 MH/s"),
                                      (16.36e9, "16.36 GH/s"), (1.3e14, "130.00 TH/s"), (2e15, "2.00 PH/s")])
def test_format_hash_rate(hps, want):
    assert tui.format_hash_rate(hps) == want


@pytest.mark.parametrize("sec,want", [(0, "0s"), (59, "59s"), (61, "1m 1s"), (3725, "1h 2m 5s")])
def test_format_duration(sec, want):
    assert tui.format_duration(sec) == want


def test_sats_to_display():
    assert tui.sats_to_display(5) == "5 sats"
    assert tui.sats_to_display(1500) == "1500 sats (0.00002 BTC)"
    assert tui.sats_to_display(150_000_000) == "1.5000 BTC"


def test_visible_len_and_truncate():
    s = tui.GREEN + "hello" + tui.RESET + "\x1b[2J!"
    assert tui.visible_len(s) == 6
    t = tui.truncate_visible(s, 3)
    assert tui.visible_len(t) == 3 and t.endswith(tui.RESET)
    assert tui.truncate_visible(s, 0) == ""
    assert tui.truncate_to_budget("abcdefgh", 5) == "ab..."
    assert tui.truncate_to_budget("abc", 2) == "ab"
    assert tui.truncate_to_budget("abc", 0) == ""
    assert tui.shorten_url("stratum+tcp://x.example:3333", 10) == "stratum..."


@pytest.mark.parametrize("cols", [40, 60, 80, 132])
def test_frame_fits_width(cols):
    d = tui.Dashboard(io.StringIO())
    d.set_width(cols)
    s = tui.Stats(hash_rate=16.36e9, shares_found=10, shares_sent=9, connected=True, pool_latency_ms=42,
                  pool_url="stratum+tls://a-very-long-pool-hostname.example.com:3333/path", devices=8,
                  devices_idle=1, wallet_fingerprint="deadbeef", uptime=3725,
                  providers=[tui.ProviderStats("mining", 1.5, True), tui.ProviderStats("akash-sim", 0.2, False)])
    frame = d.render(s)
    lines = frame.split("\r\n")[:-1]
    assert all(tui.visible_len(ln.replace(tui.HOME, "")) == cols for ln in lines)
    assert "16.36 GH/s" in frame and "ARBITRATION" in frame and "deadbeef" in frame
    assert "✓ connected" in frame


def test_status_badges():
    d = tui.Dashboard(io.StringIO())
    assert "paused" in d.mining_line(tui.Stats(curtailed=True))
    assert "stalled" in d.mining_line(tui.Stats(stalled=True))
    assert "disconnected" in d.pool_line(tui.Stats())
    assert "not initialized" in d.wallet_line(tui.Stats())


def test_set_width_floor():
    d = tui.Dashboard(io.StringIO())
    d.set_width(20)
    assert d.cols == 80


def test_loop_renders_and_stops():
    w = io.StringIO()
    d = tui.Dashboard(w, interval=0.02)
    d.start()
    d.update({"hashrate": 5e9, "connected": True, "pool": "stratum+tcp://p:3333", "devices": {"gpu-0": 5e9}})
    time.sleep(0.15)
    d.stop()
    out = w.getvalue()
    assert "5.00 GH/s" in out and out.endswith("\x1b[?25h\n")
