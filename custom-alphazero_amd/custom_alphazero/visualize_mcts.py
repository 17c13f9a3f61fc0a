"""MctsVisualizer over the device tree (reference visualize_mcts.py:7-151).

The reference renders UCTNode/UCTEdge objects with graphviz.Digraph; here the
nodes and edges are the read-only views custom_alphazero.mcts.mcts builds from
az_tree_export (the device arena), so the reference's traversal, labels and
colours apply unchanged.  graphviz is used when it is importable; otherwise a
small DOT writer stands in (graphviz is not installed in this image), which
keeps `.source`, `.save()` and `.edge()` and raises on rendering.
"""
import os

try:  # pragma: no cover - graphviz is absent here
    from graphviz import Digraph
except ImportError:  # the DOT text is all the reference's graph holds before rendering
    class Digraph:
        def __init__(self, name="G", filename=None):
            self.name = name
            self.filename = filename or f"{name}.gv"
            self.body = []

        @staticmethod
        def _q(s):
            return '"' + str(s).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n") + '"'

        def edge(self, tail, head, **attrs):
            a = " ".join(f"{k}={self._q(v)}" for k, v in attrs.items())
            self.body.append(f"\t{self._q(tail)} -> {self._q(head)} [{a}]")

        @property
        def source(self):
            return "digraph " + self.name + " {\n" + "\n".join(self.body) + "\n}\n"

        def save(self, filename=None, directory=None):
            path = os.path.join(directory or "", filename or self.filename)
            with open(path, "w") as fp:
                fp.write(self.source)
            return path

        def render(self, *args, **kwargs):
            raise RuntimeError("graphviz is not installed: use .save() for the DOT source")

        view = render


class MctsVisualizer:
    def __init__(self, mcts_root_node=None, mcts_name="mcts", show_node_index=True,
                 remove_unplayed_edge=False, is_updated=False):
        self.mcts_root_node = mcts_root_node
        self.mcts_name = mcts_name
        self.show_node_index = show_node_index
        self.remove_unplayed_edge = remove_unplayed_edge
        self.node_ref_index = {}
        self.is_updated = is_updated
        if self.mcts_root_node:
            self.edges = MctsVisualizer._breadth_first_edges(self.mcts_root_node)
            MctsVisualizer._enrich_edges(self.edges)
            self.graph_mcts = self.mcts_graph(remove_unvisited=True)

    def build_mcts_graph(self, mcts_root_node, mcts_name=None, remove_unplayed_edge=False):
        self.mcts_root_node = mcts_root_node
        self.mcts_name = mcts_name if mcts_name is not None else self.mcts_name
        self.remove_unplayed_edge = remove_unplayed_edge
        self.edges = MctsVisualizer._breadth_first_edges(self.mcts_root_node)
        MctsVisualizer._enrich_edges(self.edges)
        self.graph_mcts = self.mcts_graph(remove_unvisited=True)

    @staticmethod
    def _breadth_first_edges(root_node):
        edges, queue = [], [root_node]
        while queue:
            node = queue.pop(0)
            for edge in node.edges:
                queue.append(edge.child)
                edges.append(edge)
        return edges

    def _describe_node(self, node, round_value_at=2):
        if id(node) not in self.node_ref_index:
            self.node_ref_index[id(node)] = len(self.node_ref_index)
        text = f"node #{self.node_ref_index[id(node)]}{os.linesep}{os.linesep}" if self.show_node_index else ""
        text += node.board.repr_graphviz()
        if node.evaluated_value is not None:
            text += f"{os.linesep}{os.linesep}V={round(node.evaluated_value, round_value_at)}"
        return text

    @staticmethod
    def _describe_edge(edge):
        label = (f"UCT={edge.upper_confidence_bound():.2f} Q={edge.exploitation_term():.2f} "
                 f"U={edge.exploration_term():.2f} {os.linesep} "
                 f"P={edge.prior:.2f} N={edge.visit_count} PN={edge.proportion_n:.2f} A={edge.action}")
        return {"label": label, "color": "red" if edge.played else "black",
                "line_width": "4" if edge.greedily_played else "1"}

    @staticmethod
    def _enrich_edges(edges):
        seen = set()
        for edge in edges:
            node = edge.parent
            if id(node) in seen:
                continue
            total = sum(e.visit_count for e in node.edges)
            for e in node.edges:
                # all proportions 0 when no edge of the node was visited
                e.proportion_n = float(e.visit_count) / total if total > 0 else 0
            seen.add(id(node))

    def mcts_graph(self, remove_unvisited=True):
        edges = [e for e in self.edges if e.visit_count > 0] if remove_unvisited else self.edges
        if self.remove_unplayed_edge:
            edges = [e for e in edges if e.played]
        graph = Digraph("G", filename=f"{self.mcts_name}.gv")
        for edge in edges:
            d = MctsVisualizer._describe_edge(edge)
            graph.edge(self._describe_node(edge.parent), self._describe_node(edge.child),
                       color=d["color"], label=d["label"], penwidth=d["line_width"])
        return graph

    def save_as_pdf(self, filename=None, directory=None, remove_gv_file=True):
        if directory is not None:
            os.makedirs(directory, exist_ok=True)
        filename = filename if filename is not None else self.graph_mcts.filename
        self.graph_mcts.render(view=False, filename=filename, directory=directory)
        if remove_gv_file:
            path = filename if directory is None else os.path.join(directory, filename)
            os.remove(path)

    def show(self, filename=None, directory=None):
        self.graph_mcts.view(filename=filename, directory=directory)
