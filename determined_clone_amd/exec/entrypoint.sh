#!/bin/bash
# Task entrypoint wrapper (reference: master/static/srv/entrypoint.sh and the notebook / shell /
# tensorboard / command entrypoints): run from the task's context directory, source the user's
# startup-hook.sh if the context directory has one -- so whatever it exports, installs or
# activates is in effect for the task -- then exec the task command ("$@").
set -e
STARTUP_HOOK="startup-hook.sh"
if [ -f "${STARTUP_HOOK}" ]; then
    set -x
    source "${STARTUP_HOOK}"
    set +x
fi
exec "$@"
