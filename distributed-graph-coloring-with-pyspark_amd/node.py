"""Node data model -- same fields and (de)serialisation as the reference's node.py:1-18."""


class Node:
    def __init__(self, id, neighbors=None, color=-1):
        self.id = id
        self.neighbors = neighbors if neighbors else []
        self.color = color

    def to_dict(self):
        return {"id": self.id, "neighbors": [nb.id for nb in self.neighbors], "color": self.color}

    @staticmethod
    def from_dict(data):
        return Node(data["id"], [], data["color"])
