"""Generates tests/golden/wordcount_tokens.json: the token stream of the WindowWordCount example's default
input (BASELINE configs[0]), i.e. the lines of WordCountData.WORDS
(flink-examples/flink-examples-streaming/src/main/java/org/apache/flink/streaming/examples/wordcount/util/
WordCountData.java:27-63) tokenized exactly as WordCount.Tokenizer does (WordCount.java:107-116:
value.toLowerCase().split("\\W+"), empty tokens dropped).  Run here (where /root/reference exists); the
JSON is the committed data fixture the bench and tests read on the GPU box.
"""
import json
import os
import re

SRC = ("/root/reference/flink-examples/flink-examples-streaming/src/main/java/org/apache/flink/streaming/examples/"
       "wordcount/util/WordCountData.java")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wordcount_tokens.json")


def main():
    text = open(SRC).read()
    body = text[text.index("WORDS = new String[]"):]
    body = body[:body.index("};")]
    lines = [bytes(m, "utf-8").decode("unicode_escape") for m in re.findall(r'"((?:[^"\\]|\\.)*)"', body)]
    tokens = []
    for line in lines:
        # Java's \W is [^a-zA-Z0-9_]
        tokens += [t for t in re.split(r"[^a-zA-Z0-9_]+", line.lower()) if t]
    json.dump({"source": "WordCountData.java:27-63 tokenized as WordCount.java:107-116",
               "lines": len(lines), "tokens": tokens, "distinct": len(set(tokens))}, open(OUT, "w"), indent=0)
    print(len(lines), "lines,", len(tokens), "tokens,", len(set(tokens)), "distinct")


if __name__ == "__main__":
    main()
