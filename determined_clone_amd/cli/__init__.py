"""``det`` CLI."""
from determined_clone_amd.cli.cli import build_parser, main
