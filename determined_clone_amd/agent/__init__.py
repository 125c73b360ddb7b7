"""Agent (reference: `agent/`)."""
from determined_clone_amd.agent.agent import Agent, detect_devices
