"""Small hand-written inputs for edge-case goldens (test data)."""

INLINE = {
    "empty": "",
    "abc": "abc abc",
    "crlf": "line one\r\nline two\rline three\r\n\r\nfour  \r\n five\r",
    "aaaa": "aaaa aaaaa aa a abab ababab aaa bbb abababab a a a aaaa",
    "special_word": "the cat the hat hello there hello the the<|endoftext|> the end",
    "dup_special": "a banana and a bandana<|endoftext|>abc a b c",
    "ws_edges": "x  \n\n y\t\t\nz 　　w v \x1c u   ",
    "contractions": "don't I'm we've they're she'll he'd it's IT'S ''s 's' x'y 'll'",
}
