"""``python -m otedama_amd <command>`` — same as the ``otedama`` CLI (cmd/otedama/main.go)."""
from otedama_amd.cli.main import main

if __name__ == "__main__":
    main()
