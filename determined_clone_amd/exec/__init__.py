"""Task entrypoints run by the agent (reference: `harness/determined/exec/`)."""
