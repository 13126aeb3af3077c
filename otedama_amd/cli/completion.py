"""``otedama completion bash|zsh|fish`` (cmd/otedama/completion.go:24-40).

Scripts are generated from the command table rather than kept as static text,
so new subcommands (pool, bench, devices) complete automatically.
"""
from __future__ import annotations

from typing import TextIO

from otedama_amd.cli.main import EXIT_OK, EXIT_USAGE

SHELLS = ("bash", "zsh", "fish")
COMMANDS = {
    "run": "Start mining on MI355X GPUs / CPU",
    "node": "Run one rank per GPU (fault-tolerant RCCL node)",
    "pool": "Run the local Stratum pool",
    "bench": "Measure hash rates",
    "devices": "List mining devices",
    "version": "Print version information",
    "config": "Inspect or validate configuration",
    "service": "Install/uninstall background service",
    "doctor": "Run self-diagnostic checks",
    "help": "Print help",
    "completion": "Generate shell completion",
}
SUBCOMMANDS = {"config": "show validate", "service": "install uninstall status", "completion": "bash zsh fish",
               "node": "status"}


def join_or(items) -> str:
    items = list(items)
    if not items:
        return ""
    if len(items) == 1:
        return items[0]
    return ", ".join(items[:-1]) + " or " + items[-1]


def bash_script() -> str:
    cases = "\n".join(f'        {k}) COMPREPLY=( $(compgen -W "{v}" -- "${{cur}}") ) ;;' for k, v in SUBCOMMANDS.items())
    return f"""# bash completion for otedama
_otedama() {{
    local cur="${{COMP_WORDS[COMP_CWORD]}}"
    local commands="{' '.join(COMMANDS)}"
    if [ "${{COMP_CWORD}}" -eq 1 ]; then
        COMPREPLY=( $(compgen -W "${{commands}}" -- "${{cur}}") )
        return
    fi
    case "${{COMP_WORDS[1]}}" in
{cases}
    esac
}}
complete -F _otedama otedama
"""


def zsh_script() -> str:
    cases = "\n".join(f"        {k}) _values '{k} argument' {v} ;;" for k, v in SUBCOMMANDS.items())
    return f"""#compdef otedama
# zsh completion for otedama
_otedama() {{
    local -a commands
    commands=({' '.join(COMMANDS)})
    if (( CURRENT == 2 )); then
        _describe 'otedama command' commands
        return
    fi
    case $words[2] in
{cases}
    esac
}}
compdef _otedama otedama
"""


def fish_script() -> str:
    lines = ["# fish completion for otedama", "complete -c otedama -f"]
    lines += [f"complete -c otedama -n __fish_use_subcommand -a {k} -d '{d}'" for k, d in COMMANDS.items()]
    lines += [f"complete -c otedama -n '__fish_seen_subcommand_from {k}' -a '{v}'" for k, v in SUBCOMMANDS.items()]
    return "\n".join(lines) + "\n"


def cmd_completion(args: list[str], stdout: TextIO, stderr: TextIO) -> int:
    if len(args) != 1:
        stderr.write(f"otedama completion: expected one shell argument ({join_or(SHELLS)})\n")
        return EXIT_USAGE
    gen = {"bash": bash_script, "zsh": zsh_script, "fish": fish_script}.get(args[0])
    if gen is None:
        stderr.write(f"otedama completion: unsupported shell {args[0]!r} (want {join_or(SHELLS)})\n")
        return EXIT_USAGE
    stdout.write(gen())
    return EXIT_OK
