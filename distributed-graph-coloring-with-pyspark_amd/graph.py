"""Graph container -- the reference's graph.py:1-43 surface (generate / serialize /
deserialize), backed by gcolor_amd's generator and JSON I/O.  ``Graph(n, D)`` after
``random.seed(s)`` reproduces the reference's graph exactly."""
import json

from gcolor_amd.generators import reference_graph
from node import Node


class Graph:
    def __init__(self, node_count, max_degree):
        self.nodes = self.generate_graph(node_count, max_degree)

    def serialize_graph(self, path):
        with open(path, "w") as f:
            json.dump([node.to_dict() for node in self.nodes], f, indent=4)

    def deserialize_graph(self, path):
        with open(path, "r") as f:
            node_data = json.load(f)
        nodes = [Node(data["id"]) for data in node_data]
        node_dict = {node.id: node for node in nodes}
        for node, data in zip(nodes, node_data):
            node.neighbors = [node_dict[nid] for nid in data["neighbors"]]
        self.nodes = nodes
        return nodes

    def generate_graph(self, node_count, max_degree):
        adj = reference_graph(node_count, max_degree)
        nodes = [Node(i) for i in range(node_count)]
        for nd, nb in zip(nodes, adj):
            nd.neighbors = [nodes[u] for u in nb]
        return nodes
