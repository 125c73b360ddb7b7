"""Master: REST API, experiments/trials, searcher driving, resource manager, persistence."""
from determined_clone_amd.master.core import Master
from determined_clone_amd.master.server import MasterServer
