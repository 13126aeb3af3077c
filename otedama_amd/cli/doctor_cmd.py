"""``otedama doctor`` (cmd/otedama/doctor.go:16-47): exit 0 pass / 1 warn / 2 fail."""
from __future__ import annotations

from typing import TextIO

from otedama_amd.cli.flags import FlagSet
from otedama_amd.cli.main import parse_subcommand


def cmd_doctor(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    from otedama_amd import config as C
    from otedama_amd import doctor

    fs = FlagSet("doctor", stderr)
    fs.string("config", "", "Path to config.yaml to diagnose.")
    fs.string("bitcoin-address", "", "Bitcoin address to validate.")
    fs.string("data-dir", "", "Data directory to check.")
    fs.bool("json", False, "Emit results as a JSON object (for CI/monitoring) instead of text.")
    rc = parse_subcommand(fs, args, stdout, stderr)
    if rc is not None:
        return rc
    path = fs["config"] or C.default_config_path()
    file_cfg, warn = C.load_config_file(path)
    if warn:
        stderr.write(f"warning: {warn}\n")
    cfg = C.resolve(file_cfg, None, C.FlagValues(bitcoin_address=fs["bitcoin-address"], data_dir=fs["data-dir"]))
    # The reference passes only --config to the Configuration check, so a default config file that exists is
    # reported as "no config file found"; here the file actually loaded is the one diagnosed.
    import os

    diagnosed = fs["config"] or (path if path and os.path.exists(path) else "")
    report = doctor.Runner(doctor.default_checks(cfg, diagnosed), timeout=30.0).run()
    if fs["json"]:
        report.write_json(stdout)
    else:
        report.print(stdout)
    return report.exit_code()
