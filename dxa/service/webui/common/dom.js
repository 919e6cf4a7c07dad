// DOM helpers shared by every package (the role React + Office Fabric play in the reference's datax-common).
// No framework: components are functions returning elements; state lives in plain objects and a component
// re-renders itself by replacing its root element's children.

export function h(tag, attrs, ...children) {
    const el = document.createElement(tag);
    if (attrs) {
        for (const k of Object.keys(attrs)) {
            const v = attrs[k];
            if (v === undefined || v === null || v === false) continue;
            if (k.startsWith('on') && typeof v === 'function') el.addEventListener(k.slice(2).toLowerCase(), v);
            else if (k === 'class') el.className = v;
            else if (k === 'style' && typeof v === 'object') Object.assign(el.style, v);
            else if (k === 'value') el.value = v;
            else if (k === 'checked') el.checked = !!v;
            else if (k === 'disabled') el.disabled = !!v;
            else el.setAttribute(k, v === true ? '' : String(v));
        }
    }
    append(el, children);
    return el;
}

function append(el, children) {
    for (const c of children) {
        if (c === undefined || c === null || c === false) continue;
        if (Array.isArray(c)) append(el, c);
        else if (typeof c === 'string' || typeof c === 'number') el.appendChild(document.createTextNode(String(c)));
        else el.appendChild(c);
    }
}

export function clear(el) {
    while (el.firstChild) el.removeChild(el.firstChild);
    return el;
}

export function mount(el, ...children) {
    clear(el);
    append(el, children);
    return el;
}

export const svgNS = 'http://www.w3.org/2000/svg';

export function s(tag, attrs, ...children) {
    const el = document.createElementNS(svgNS, tag);
    if (attrs) for (const k of Object.keys(attrs)) if (attrs[k] !== undefined && attrs[k] !== null) el.setAttribute(k, String(attrs[k]));
    const add = cs => {
        for (const c of cs) {
            if (c === undefined || c === null || c === false) continue;
            if (Array.isArray(c)) add(c);
            else el.appendChild(typeof c === 'string' || typeof c === 'number' ? document.createTextNode(String(c)) : c);
        }
    };
    add(children);
    return el;
}

export function deepClone(o) {
    return o === undefined ? undefined : JSON.parse(JSON.stringify(o));
}

// number formatting used by the metric widgets (the reference's d3-format based formatterDict)
export const formatters = {
    identical: d => String(d),
    longint: d => (isNaN(d) ? '-' : Math.round(d).toLocaleString('en-US')),
    int: d => (isNaN(d) ? '-' : String(Math.round(d))),
    floatNumber: d => (isNaN(d) ? '-' : String(Math.floor(d * 100) / 100)),
    percentage: d => (isNaN(d) ? '-' : Math.floor(d * 100 * 1000) / 1000 + '%'),
    si: d => {
        if (isNaN(d)) return '-';
        const a = Math.abs(d);
        const units = [[1e12, 'T'], [1e9, 'G'], [1e6, 'M'], [1e3, 'k']];
        for (const [v, u] of units) if (a >= v) return (d / v).toFixed(a / v >= 100 ? 0 : 1) + u;
        return String(Math.round(d * 100) / 100);
    }
};

export function formatTime(t) {
    const d = t instanceof Date ? t : new Date(t);
    const p = n => String(n).padStart(2, '0');
    return `${p(d.getHours())}:${p(d.getMinutes())}:${p(d.getSeconds())}`;
}
