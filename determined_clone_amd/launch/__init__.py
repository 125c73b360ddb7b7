"""Launch layers (reference: `harness/determined/launch/`)."""
