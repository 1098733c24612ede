import pstats,sys
p=pstats.Stats(sys.argv[1]); p.sort_stats('tottime').print_stats(30)
