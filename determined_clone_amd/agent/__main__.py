from determined_clone_amd.agent.agent import main

main()
