"""Hyperparameter search (reference: `master/pkg/searcher`, `harness/determined/searcher`).

Master-side search methods live in :mod:`.methods` (``methods.SearchMethod`` is their base class);
the user-facing custom-searcher API (``SearchMethod``, ``SearcherState``, ``LocalSearchRunner``,
``RemoteSearchRunner``, ``Progress``) mirrors ``determined.searcher``.
"""
from determined_clone_amd.searcher.methods import (AdaptiveASHASearch, AsyncHalvingSearch,
                                                   AsyncHalvingStoppingSearch, Close, Context,
                                                   Create, CustomSearch, GridSearch, Operation,
                                                   RandomSearch, Shutdown, SingleSearch,
                                                   TournamentSearch, ValidateAfter,
                                                   make_search_method, op_from_dict)
from determined_clone_amd.searcher.methods import SearchMethod as MasterSearchMethod
from determined_clone_amd.searcher.custom import (ExitedReason, LocalSearchRunner, Progress,
                                                  RemoteSearchRunner, SearcherState, SearchMethod,
                                                  SearchRunner)
from determined_clone_amd.searcher._searcher import Searcher
from determined_clone_amd.searcher.simulate import (constant_validation, random_validation,
                                                    simulate, trial_id_metric)
from determined_clone_amd.searcher import hparams
