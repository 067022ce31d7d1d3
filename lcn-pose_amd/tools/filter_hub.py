"""Skeleton adjacency of the 17-joint H36M layout (tools/filter_hub.py:4-24 of
the reference): joint -> neighbouring joints."""

neighbour_dict_set = [
    {0: [1, 4, 7],
     1: [0, 7, 2],
     2: [1, 3],
     3: [2],
     4: [0, 7, 5],
     5: [4, 6],
     6: [5],
     7: [1, 0, 4, 14, 8, 11],
     8: [7, 9, 11, 14],
     9: [8, 10],
     10: [9],
     11: [8, 7, 12],
     12: [11, 13],
     13: [12],
     14: [8, 7, 15],
     15: [14, 16],
     16: [15]},
]
