from .agent import main

main()
