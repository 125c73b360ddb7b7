"""Hyperparameter search (reference: `master/pkg/searcher`, `harness/determined/searcher`)."""
from determined_clone_amd.searcher.methods import (AdaptiveASHASearch, AsyncHalvingSearch,
                                                   AsyncHalvingStoppingSearch, Close, Context,
                                                   Create, CustomSearch, ExitedReason, GridSearch,
                                                   Operation, RandomSearch, SearchMethod, Shutdown,
                                                   SingleSearch, TournamentSearch, ValidateAfter,
                                                   make_search_method, op_from_dict)
from determined_clone_amd.searcher._searcher import Searcher
from determined_clone_amd.searcher.simulate import (constant_validation, random_validation,
                                                    simulate, trial_id_metric)
from determined_clone_amd.searcher import hparams
